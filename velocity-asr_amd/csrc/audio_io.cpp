// Host-side audio I/O behind load_audio (reference velocity_asr/audio.py:22-62): a FLAC
// stream decoder (torchaudio.load's format for LibriSpeech, audio.py:47) and the windowed-sinc
// resampler of torchaudio.transforms.Resample (audio.py:54-56) with its default parameters.
// Both run on the host: they turn files into the (channels, samples) float32 waveform that the
// HIP front end consumes; nothing here is on the device path.
//
// FLAC (the format specification, RFC 9639): "fLaC", metadata blocks (STREAMINFO required,
// others skipped; an ID3v2 tag in front is skipped), then frames: a sync'd header (CRC-8), one
// subframe per channel (CONSTANT, VERBATIM, FIXED order 0-4, LPC order 1-32; wasted bits; Rice
// or Rice2 residual with partitions and escape codes), inter-channel decorrelation (left/side,
// side/right, mid/side) and a CRC-16 footer.  Samples are scaled to [-1, 1) by 2^(bps-1), as
// torchaudio.load normalises integer PCM.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <exception>
#include <vector>

#include "vasr_internal.h"

namespace vasr {
namespace {

struct BitReader {
    const uint8_t* p;
    int64_t n;      // bytes
    int64_t pos;    // bit position
    bool overrun = false;

    uint32_t bit() {
        if (pos >= n * 8) {
            overrun = true;
            return 0;
        }
        const uint32_t b = (p[pos >> 3] >> (7 - (pos & 7))) & 1u;
        ++pos;
        return b;
    }
    uint64_t bits(int k) {  // k <= 64
        uint64_t v = 0;
        // fast path: byte aligned whole bytes
        while (k >= 8 && (pos & 7) == 0 && pos / 8 < n) {
            v = (v << 8) | p[pos >> 3];
            pos += 8;
            k -= 8;
        }
        while (k-- > 0) v = (v << 1) | bit();
        return v;
    }
    int64_t sbits(int k) {
        if (k == 0) return 0;
        const uint64_t u = bits(k);
        const uint64_t sign = 1ull << (k - 1);
        return (int64_t)(u ^ sign) - (int64_t)sign;
    }
    uint32_t unary() {  // number of 0 bits before the next 1
        uint32_t c = 0;
        while (!overrun) {
            if ((pos & 7) == 0 && pos / 8 < n && p[pos >> 3] == 0) {
                c += 8;
                pos += 8;
                continue;
            }
            if (bit()) break;
            ++c;
        }
        return c;
    }
    void align() { pos = (pos + 7) & ~(int64_t)7; }
};

uint8_t crc8(const uint8_t* d, int64_t n) {
    uint8_t c = 0;
    for (int64_t i = 0; i < n; ++i) {
        c ^= d[i];
        for (int b = 0; b < 8; ++b) c = (uint8_t)((c & 0x80) ? (c << 1) ^ 0x07 : c << 1);
    }
    return c;
}

uint16_t crc16(const uint8_t* d, int64_t n) {
    uint16_t c = 0;
    for (int64_t i = 0; i < n; ++i) {
        c ^= (uint16_t)d[i] << 8;
        for (int b = 0; b < 8; ++b) c = (uint16_t)((c & 0x8000) ? (c << 1) ^ 0x8005 : c << 1);
    }
    return c;
}

struct StreamInfo {
    int sample_rate = 0, channels = 0, bps = 0;
    int64_t total = 0;
    int64_t first_frame = 0;  // byte offset of the first frame
};

bool parse_header(const uint8_t* d, int64_t n, StreamInfo& si, const char*& err) {
    int64_t off = 0;
    if (n >= 10 && std::memcmp(d, "ID3", 3) == 0) {  // ID3v2 tag: 10-byte header + syncsafe size
        const int64_t sz = ((int64_t)(d[6] & 0x7F) << 21) | ((d[7] & 0x7F) << 14) | ((d[8] & 0x7F) << 7) | (d[9] & 0x7F);
        off = 10 + sz + ((d[5] & 0x10) ? 10 : 0);
    }
    if (n < off + 4 || std::memcmp(d + off, "fLaC", 4) != 0) {
        err = "not a FLAC stream (no fLaC marker)";
        return false;
    }
    off += 4;
    bool have_info = false;
    for (;;) {
        if (off + 4 > n) {
            err = "truncated metadata";
            return false;
        }
        const bool last = d[off] & 0x80;
        const int type = d[off] & 0x7F;
        const int64_t len = ((int64_t)d[off + 1] << 16) | (d[off + 2] << 8) | d[off + 3];
        off += 4;
        if (off + len > n) {
            err = "truncated metadata block";
            return false;
        }
        if (type == 0) {
            if (len < 34) {
                err = "short STREAMINFO";
                return false;
            }
            BitReader br{d + off, len, 0};
            br.bits(16);  // min block size
            br.bits(16);  // max block size
            br.bits(24);  // min frame size
            br.bits(24);  // max frame size
            si.sample_rate = (int)br.bits(20);
            si.channels = (int)br.bits(3) + 1;
            si.bps = (int)br.bits(5) + 1;
            si.total = (int64_t)br.bits(36);
            have_info = true;
        }
        off += len;
        if (last) break;
    }
    if (!have_info) {
        err = "no STREAMINFO block";
        return false;
    }
    si.first_frame = off;
    return true;
}

// Residual of one subframe into res[order .. bs).
bool read_residual(BitReader& br, int bs, int order, int32_t* res, const char*& err) {
    const int method = (int)br.bits(2);
    if (method > 1) {
        err = "reserved residual coding method";
        return false;
    }
    const int pbits = method == 0 ? 4 : 5;
    const uint32_t escape = method == 0 ? 15u : 31u;
    const int porder = (int)br.bits(4);
    const int parts = 1 << porder;
    if ((bs >> porder) << porder != bs || (bs >> porder) < order) {
        err = "bad residual partition order";
        return false;
    }
    int i = order;
    for (int pt = 0; pt < parts; ++pt) {
        const int cnt = (bs >> porder) - (pt == 0 ? order : 0);
        const uint32_t k = (uint32_t)br.bits(pbits);
        if (k == escape) {
            const int nb = (int)br.bits(5);
            for (int j = 0; j < cnt; ++j) res[i++] = (int32_t)br.sbits(nb);
        } else {
            for (int j = 0; j < cnt; ++j) {
                const uint64_t q = br.unary();
                const uint64_t u = (q << k) | br.bits((int)k);
                res[i++] = (int32_t)((int64_t)(u >> 1) ^ -(int64_t)(u & 1));
            }
        }
        if (br.overrun) {
            err = "truncated residual";
            return false;
        }
    }
    return true;
}

// A decoded sample must fit the subframe's sample size; a corrupt residual that does not would
// feed ever-growing values into the predictors (and, at 32 taps of 15-bit coefficients, overflow
// their int64 sums), so it ends the decode instead.
inline bool fits(int64_t v, int bps) { return v >= -((int64_t)1 << (bps - 1)) && v < ((int64_t)1 << (bps - 1)); }

bool read_subframe(BitReader& br, int bs, int bps, int64_t* out, std::vector<int32_t>& res, const char*& err) {
    if (br.bit() != 0) {
        err = "subframe padding bit set";
        return false;
    }
    const int type = (int)br.bits(6);
    int wasted = 0;
    if (br.bit()) wasted = (int)br.unary() + 1;
    bps -= wasted;
    if (bps <= 0 || bps > 33) {
        err = "bad subframe sample size";
        return false;
    }
    if (type == 0) {  // CONSTANT
        const int64_t v = br.sbits(bps);
        for (int i = 0; i < bs; ++i) out[i] = v;
    } else if (type == 1) {  // VERBATIM
        for (int i = 0; i < bs; ++i) out[i] = br.sbits(bps);
    } else if (type >= 8 && type <= 12) {  // FIXED
        const int order = type - 8;
        if (order > bs) {
            err = "fixed order exceeds block";
            return false;
        }
        for (int i = 0; i < order; ++i) out[i] = br.sbits(bps);
        res.resize(bs);
        if (!read_residual(br, bs, order, res.data(), err)) return false;
        for (int i = order; i < bs; ++i) {
            int64_t pred = 0;
            switch (order) {
                case 1: pred = out[i - 1]; break;
                case 2: pred = 2 * out[i - 1] - out[i - 2]; break;
                case 3: pred = 3 * out[i - 1] - 3 * out[i - 2] + out[i - 3]; break;
                case 4: pred = 4 * out[i - 1] - 6 * out[i - 2] + 4 * out[i - 3] - out[i - 4]; break;
                default: break;
            }
            out[i] = pred + res[i];
            if (!fits(out[i], bps)) {
                err = "fixed-predictor sample exceeds the sample size";
                return false;
            }
        }
    } else if (type >= 32) {  // LPC
        const int order = type - 31;
        if (order > bs) {
            err = "lpc order exceeds block";
            return false;
        }
        for (int i = 0; i < order; ++i) out[i] = br.sbits(bps);
        const int prec = (int)br.bits(4) + 1;
        if (prec == 16) {
            err = "invalid LPC coefficient precision";
            return false;
        }
        const int shift = (int)br.sbits(5);
        if (shift < 0) {
            err = "negative LPC shift";
            return false;
        }
        int64_t coef[32];
        for (int j = 0; j < order; ++j) coef[j] = br.sbits(prec);
        res.resize(bs);
        if (!read_residual(br, bs, order, res.data(), err)) return false;
        for (int i = order; i < bs; ++i) {
            int64_t acc = 0;
            for (int j = 0; j < order; ++j) acc += coef[j] * out[i - 1 - j];
            out[i] = (acc >> shift) + res[i];
            if (!fits(out[i], bps)) {
                err = "LPC sample exceeds the sample size";
                return false;
            }
        }
    } else {
        err = "reserved subframe type";
        return false;
    }
    if (br.overrun) {
        err = "truncated subframe";
        return false;
    }
    if (wasted)
        for (int i = 0; i < bs; ++i) out[i] = (int64_t)((uint64_t)out[i] << wasted);
    return true;
}

// Per-channel cap on decoded samples (2^28: 4.6 h at 16 kHz, 2 GiB of int64 per channel).
constexpr int64_t kMaxFlacSamples = (int64_t)1 << 28;

// Decode every frame; samples[c] grows per channel.
bool decode_frames(const uint8_t* d, int64_t n, const StreamInfo& si, std::vector<std::vector<int64_t>>& samples,
                   int& bps_out, const char*& err) {
    static const int kRates[12] = {0, 88200, 176400, 192000, 8000, 16000, 22050, 24000, 32000, 44100, 48000, 96000};
    static const int kBits[8] = {0, 8, 12, -1, 16, 20, 24, 32};
    samples.assign(si.channels, {});
    std::vector<int64_t> sub[8];
    std::vector<int32_t> res;
    bps_out = si.bps;
    int64_t off = si.first_frame;
    while (off + 2 <= n) {
        if (!(d[off] == 0xFF && (d[off + 1] & 0xFE) == 0xF8)) {
            if (si.total > 0 && (int64_t)samples[0].size() >= si.total) break;  // trailing tag / padding
            err = "lost frame sync";
            return false;
        }
        BitReader br{d + off, n - off, 16};
        const int bs_code = (int)br.bits(4), sr_code = (int)br.bits(4);
        const int ch_code = (int)br.bits(4), sz_code = (int)br.bits(3);
        if (br.bit() != 0) {
            err = "reserved frame header bit set";
            return false;
        }
        // coded frame / sample number (UTF-8-like, up to 7 bytes)
        const uint32_t b0 = (uint32_t)br.bits(8);
        int extra = 0;
        if (b0 & 0x80) {
            uint32_t m = 0x40;
            while (b0 & m) {
                ++extra;
                m >>= 1;
            }
            if (extra < 1 || extra > 6) {
                err = "bad frame number coding";
                return false;
            }
            for (int i = 0; i < extra; ++i) br.bits(8);
        }
        int bs;
        if (bs_code == 0) {
            err = "reserved block size code";
            return false;
        } else if (bs_code == 1) {
            bs = 192;
        } else if (bs_code <= 5) {
            bs = 576 << (bs_code - 2);
        } else if (bs_code == 6) {
            bs = (int)br.bits(8) + 1;
        } else if (bs_code == 7) {
            bs = (int)br.bits(16) + 1;
        } else {
            bs = 256 << (bs_code - 8);
        }
        if (sr_code == 12) br.bits(8);
        else if (sr_code == 13 || sr_code == 14) br.bits(16);
        else if (sr_code == 15) {
            err = "invalid sample rate code";
            return false;
        }
        (void)kRates;
        const int bps = sz_code == 0 ? si.bps : kBits[sz_code];
        if (bps <= 0) {
            err = "reserved sample size code";
            return false;
        }
        if (bps != si.bps) {  // one scale for the whole stream (vasr_flac_decode divides by 2^(bps-1))
            err = "frame sample size differs from STREAMINFO";
            return false;
        }
        const int64_t hdr_bytes = br.pos / 8;
        const uint8_t hcrc = (uint8_t)br.bits(8);
        if (br.overrun || crc8(d + off, hdr_bytes) != hcrc) {
            err = "frame header CRC-8 mismatch";
            return false;
        }
        int nch;
        if (ch_code <= 7) nch = ch_code + 1;
        else if (ch_code <= 10) nch = 2;
        else {
            err = "reserved channel assignment";
            return false;
        }
        if (nch != si.channels) {
            err = "frame channel count differs from STREAMINFO";
            return false;
        }
        for (int c = 0; c < nch; ++c) {
            const bool side = (ch_code == 8 && c == 1) || (ch_code == 9 && c == 0) || (ch_code == 10 && c == 1);
            sub[c].resize(bs);
            if (!read_subframe(br, bs, bps + (side ? 1 : 0), sub[c].data(), res, err)) return false;
        }
        br.align();
        const int64_t body = br.pos / 8;
        const uint16_t fcrc = (uint16_t)br.bits(16);
        if (br.overrun || crc16(d + off, body) != fcrc) {
            err = "frame CRC-16 mismatch";
            return false;
        }
        for (int i = 0; i < bs; ++i) {
            if (ch_code == 8) {         // left / side
                sub[1][i] = sub[0][i] - sub[1][i];
            } else if (ch_code == 9) {  // side / right
                sub[0][i] = sub[0][i] + sub[1][i];
            } else if (ch_code == 10) {  // mid / side
                const int64_t side = sub[1][i];
                const int64_t mid = (int64_t)((uint64_t)sub[0][i] << 1) | (side & 1);
                sub[0][i] = (mid + side) >> 1;
                sub[1][i] = (mid - side) >> 1;
            }
        }
        if ((int64_t)samples[0].size() + bs > kMaxFlacSamples) {
            err = "stream exceeds the decoder's sample limit";
            return false;
        }
        for (int c = 0; c < nch; ++c) samples[c].insert(samples[c].end(), sub[c].begin(), sub[c].begin() + bs);
        off += body + 2;
    }
    if (si.total > 0 && (int64_t)samples[0].size() > si.total)
        for (auto& s : samples) s.resize(si.total);
    return true;
}

}  // namespace
}  // namespace vasr

namespace {
int flac_decode(const uint8_t* data, int64_t n, float* out, int64_t out_cap, int* channels, int* sample_rate, int* bits,
                int64_t* samples) {
    using namespace vasr;
    VASR_CHECK_ARG(data && n > 0 && channels && sample_rate && bits && samples, "vasr_flac_decode: null argument");
    StreamInfo si;
    const char* err = "";
    if (!parse_header(data, n, si, err)) {
        set_error("vasr_flac_decode: %s", err);
        return VASR_EINVAL;
    }
    std::vector<std::vector<int64_t>> pcm;
    int bps = si.bps;
    if (bps < 4 || bps > 32) {
        set_error("vasr_flac_decode: STREAMINFO sample size %d outside 4..32", bps);
        return VASR_EINVAL;
    }
    if (!decode_frames(data, n, si, pcm, bps, err)) {
        set_error("vasr_flac_decode: %s", err);
        return VASR_EINVAL;
    }
    const int64_t ns = pcm.empty() ? 0 : (int64_t)pcm[0].size();
    *channels = si.channels;
    *sample_rate = si.sample_rate;
    *bits = bps;
    *samples = ns;
    if (out == nullptr) return VASR_OK;  // size query
    VASR_CHECK_ARG(out_cap >= ns * si.channels, "vasr_flac_decode: output of %lld floats, %lld needed",
                   (long long)out_cap, (long long)(ns * si.channels));
    const double scale = 1.0 / (double)(1ull << (bps - 1));
    for (int c = 0; c < si.channels; ++c)
        for (int64_t i = 0; i < ns; ++i) out[c * ns + i] = (float)((double)pcm[c][i] * scale);
    return VASR_OK;
}
}  // namespace

// The host entry points allocate (decoded PCM, resampling kernels): no exception crosses the C ABI.
VASR_API int vasr_flac_decode(const uint8_t* data, int64_t n, float* out, int64_t out_cap, int* channels,
                              int* sample_rate, int* bits, int64_t* samples) {
    try {
        return flac_decode(data, n, out, out_cap, channels, sample_rate, bits, samples);
    } catch (const std::exception& e) {
        vasr::set_error("vasr_flac_decode: %s", e.what());
        return VASR_EINVAL;
    }
}

// torchaudio.functional.resample with Resample()'s defaults (sinc_interp_hann, lowpass filter
// width 6, rolloff 0.99): per (orig, new) reduced by their gcd, a (new, 2*width + orig) kernel
// built in float64 and rounded to float32, applied as a stride-`orig` convolution over the
// signal padded by (width, width + orig) zeros; ceil(new * n / orig) outputs.  Accumulation here
// is in float64 (torch's float32 conv1d sums in its own order: equal to ~1e-7, unpinned).
VASR_API int64_t vasr_resample_length(int64_t n, int orig_sr, int new_sr) {
    if (n <= 0 || orig_sr <= 0 || new_sr <= 0) return 0;
    int64_t a = orig_sr, b = new_sr;
    while (b) {
        const int64_t t = a % b;
        a = b;
        b = t;
    }
    const int64_t o = orig_sr / a, w = new_sr / a;
    return (w * n + o - 1) / o;
}

namespace {
int resample_f32(const float* x, int channels, int64_t n, int64_t ld_x, int orig_sr, int new_sr, float* y, int64_t ld_y) {
    using namespace vasr;
    VASR_CHECK_ARG(x && y && channels > 0 && n > 0 && orig_sr > 0 && new_sr > 0 && ld_x >= n,
                   "vasr_resample_f32: bad arguments");
    int64_t g = orig_sr, r = new_sr;
    while (r) {
        const int64_t t = g % r;
        g = r;
        r = t;
    }
    const int orig = (int)(orig_sr / g), nw = (int)(new_sr / g);
    const int64_t out_len = vasr_resample_length(n, orig_sr, new_sr);
    VASR_CHECK_ARG(ld_y >= out_len, "vasr_resample_f32: ld_y %lld < %lld outputs", (long long)ld_y, (long long)out_len);
    if (orig == nw) {
        for (int c = 0; c < channels; ++c) std::memcpy(y + c * ld_y, x + c * ld_x, sizeof(float) * n);
        return VASR_OK;
    }
    const double lpw = 6.0, rolloff = 0.99;
    const double base = (double)(orig < nw ? orig : nw) * rolloff;
    const int width = (int)std::ceil(lpw * orig / base);
    const int klen = 2 * width + orig;
    // (new, 2 * width + orig) taps after the gcd reduction: rates with a small gcd (44101 -> 16000)
    // would need gigabytes of kernel
    VASR_CHECK_ARG((int64_t)nw * klen <= ((int64_t)1 << 24),
                   "vasr_resample_f32: %d -> %d Hz needs a %lld-tap kernel (limit 2^24)", orig_sr, new_sr,
                   (long long)nw * klen);
    std::vector<float> kern((size_t)nw * klen);
    const double pi = 3.14159265358979323846;
    for (int j = 0; j < nw; ++j) {
        for (int k = 0; k < klen; ++k) {
            // t = (-j / new + (k - width) / orig) * base, clamped to [-lpw, lpw]
            double t = ((double)(-j) / nw + (double)(k - width) / orig) * base;
            t = t < -lpw ? -lpw : (t > lpw ? lpw : t);
            const double c = std::cos(t * pi / lpw / 2.0);
            const double window = c * c;
            const double tp = t * pi;
            const double s = tp == 0.0 ? 1.0 : std::sin(tp) / tp;
            kern[(size_t)j * klen + k] = (float)(s * (window * (base / orig)));
        }
    }
    for (int c = 0; c < channels; ++c) {
        const float* xc = x + c * ld_x;
        float* yc = y + c * ld_y;
        for (int64_t o = 0; o < out_len; ++o) {
            const int64_t fr = o / nw;
            const int j = (int)(o - fr * nw);
            const int64_t start = fr * orig - width;  // index of kernel tap 0 in the unpadded signal
            const float* kj = kern.data() + (size_t)j * klen;
            double acc = 0.0;
            const int k0 = start < 0 ? (int)-start : 0;
            const int k1 = start + klen > n ? (int)(n - start) : klen;
            for (int k = k0; k < k1; ++k) acc += (double)kj[k] * (double)xc[start + k];
            yc[o] = (float)acc;
        }
    }
    return VASR_OK;
}
}  // namespace

VASR_API int vasr_resample_f32(const float* x, int channels, int64_t n, int64_t ld_x, int orig_sr, int new_sr, float* y,
                               int64_t ld_y) {
    try {
        return resample_f32(x, channels, n, ld_x, orig_sr, new_sr, y, ld_y);
    } catch (const std::exception& e) {
        vasr::set_error("vasr_resample_f32: %s", e.what());
        return VASR_EINVAL;
    }
}
