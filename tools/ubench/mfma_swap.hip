// Does v_mfma_f32_32x32x16_bf16 give bitwise the same C^T when the operands are swapped?
// acc1 = A x B (lane l holds B[k][l%32] / A[l%32][k]), acc2 = B^T x A^T with the same registers
// swapped; element (i, j) of acc1 must equal element (j, i) of acc2.  Chains of 6 products with
// a nonzero start accumulator, as the split-bf16 engines run them.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

__global__ void k(const unsigned short* a, const unsigned short* b, const float* c0, float* o1, float* o2, int steps) {
    const int l = threadIdx.x;
    floatx16 acc1, acc2;
    for (int i = 0; i < 16; ++i) acc1[i] = acc2[i] = c0[l * 16 + i];
    for (int s = 0; s < steps; ++s) {
        bf16x8 fa, fb;
        for (int j = 0; j < 8; ++j) {
            unsigned short ua = a[(s * 64 + l) * 8 + j], ub = b[(s * 64 + l) * 8 + j];
            fa[j] = __builtin_bit_cast(__bf16, ua);
            fb[j] = __builtin_bit_cast(__bf16, ub);
        }
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, acc1, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb, fa, acc2, 0, 0, 0);
    }
    for (int i = 0; i < 16; ++i) {
        o1[l * 16 + i] = acc1[i];
        o2[l * 16 + i] = acc2[i];
    }
}

int main() {
    const int steps = 6, trials = 200;
    int bad = 0;
    srand(1);
    unsigned short *da, *db;
    float *dc, *do1, *do2;
    (void)hipMalloc(&da, steps * 512 * 2);
    (void)hipMalloc(&db, steps * 512 * 2);
    (void)hipMalloc(&dc, 1024 * 4);
    (void)hipMalloc(&do1, 1024 * 4);
    (void)hipMalloc(&do2, 1024 * 4);
    static unsigned short a[6 * 512], b[6 * 512];
    static float c0[1024], c0b[1024], o1[1024], o2[1024];
    for (int t = 0; t < trials; ++t) {
        for (int i = 0; i < steps * 512; ++i) {
            float fa = ((rand() % 20001) - 10000) / 977.0f * (1 << (rand() % 12)) / 64.0f;
            float fb = ((rand() % 20001) - 10000) / 613.0f * (1 << (rand() % 12)) / 64.0f;
            unsigned ua, ub;
            memcpy(&ua, &fa, 4);
            memcpy(&ub, &fb, 4);
            a[i] = ua >> 16;
            b[i] = ub >> 16;
        }
        float cm[32][32];
        for (int i = 0; i < 32; ++i)
            for (int j = 0; j < 32; ++j) cm[i][j] = ((rand() % 2001) - 1000) / 37.0f;
        for (int l = 0; l < 64; ++l)
            for (int s2 = 0; s2 < 16; ++s2) {
                const int r = 8 * (s2 / 4) + 4 * (l / 32) + s2 % 4, c = l % 32;
                c0[l * 16 + s2] = cm[r][c];
                c0b[l * 16 + s2] = cm[c][r];
            }
        (void)hipMemcpy(da, a, sizeof(a), hipMemcpyHostToDevice);
        (void)hipMemcpy(db, b, sizeof(b), hipMemcpyHostToDevice);
        // acc1 = C + A B (start C)
        (void)hipMemcpy(dc, c0, sizeof(c0), hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, dc, do1, do2, steps);
        (void)hipMemcpy(o1, do1, sizeof(o1), hipMemcpyDeviceToHost);
        float r1[32][32];
        for (int l = 0; l < 64; ++l)
            for (int s2 = 0; s2 < 16; ++s2) r1[8 * (s2 / 4) + 4 * (l / 32) + s2 % 4][l % 32] = o1[l * 16 + s2];
        // acc2 = C^T + (A B)^T with the operands swapped (start C^T)
        (void)hipMemcpy(dc, c0b, sizeof(c0b), hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, dc, do1, do2, steps);
        (void)hipMemcpy(o2, do2, sizeof(o2), hipMemcpyDeviceToHost);
        for (int l = 0; l < 64; ++l)
            for (int s2 = 0; s2 < 16; ++s2) {
                const int r = 8 * (s2 / 4) + 4 * (l / 32) + s2 % 4, c = l % 32;
                unsigned x, y;
                memcpy(&x, &o2[l * 16 + s2], 4);
                memcpy(&y, &r1[c][r], 4);
                if (x != y) ++bad;
            }
    }
    printf("mfma operand swap: %d of %d elements differ bitwise\n", bad, trials * 1024);
    return 0;
}
