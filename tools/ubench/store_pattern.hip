// Microbenchmark (diagnostic): HBM write bandwidth of the composed projection GEMM's output
// pattern (gemm_rows.hip's epilogue: 32 x 32 MFMA accumulator chunks, each store instruction two
// rows x 128 B of an (M, 1280) fp32 row-major C) against other layouts of the same 40 MB:
//   0 row-major, the rows engine's order (block = 256 rows x 160 columns, 8 waves x 32 rows,
//     5 chunks of 32 columns, 16 stores per chunk)
//   1 the same with non-temporal stores (the engine's cache policy)
//   2 channel-blocked [col / 16][row][col % 16]: a chunk is two contiguous 2 KB runs
//   3 contiguous: each store instruction writes 256 B, a wave's chunk 4 KB in one run
// Build: hipcc --offload-arch=gfx950 -O3 store_pattern.hip -o store_pattern
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int M = 8192, N = 1280, ROWS_PB = 256, COLS_PG = 160;

template <int PAT>
__global__ __launch_bounds__(512) void k(float* __restrict__ c, float v0) {
    const int rb = blockIdx.x / (N / COLS_PG), cg = blockIdx.x % (N / COLS_PG);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
    const int m0 = rb * ROWS_PB + wave * 32;
    for (int ch = 0; ch < COLS_PG / 32; ++ch) {
        const int n0 = cg * COLS_PG + ch * 32;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float v = v0 + i;
            if constexpr (PAT <= 1) {
                const int row = m0 + (i & 3) + 8 * (i >> 2) + 4 * h, col = n0 + r;
                float* p = c + (size_t)row * N + col;
                if constexpr (PAT == 1) __builtin_nontemporal_store(v, p);
                else *p = v;
            } else if constexpr (PAT == 2) {
                const int row = m0 + (i & 3) + 8 * (i >> 2) + 4 * h, col = n0 + r;
                c[((size_t)(col >> 4) * M + row) * 16 + (col & 15)] = v;
            } else {
                // the wave's 4 KB chunk as one run: instruction i covers floats [64 i, 64 i + 64)
                const size_t base = ((size_t)blockIdx.x * 8 + wave) * (COLS_PG / 32) * 1024 + (size_t)ch * 1024;
                c[base + i * 64 + lane] = v;
            }
        }
    }
}

template <int PAT>
float run(float* c) {
    const int grid = (M / ROWS_PB) * (N / COLS_PG);
    hipLaunchKernelGGL(k<PAT>, dim3(grid), dim3(512), 0, 0, c, 1.0f);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    const int reps = 50;
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k<PAT>, dim3(grid), dim3(512), 0, 0, c, (float)i);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms * 1e3f / reps;
}

int main() {
    float* c;
    hipMalloc(&c, (size_t)M * N * sizeof(float));
    const char* names[4] = {"row-major (rows engine order)", "row-major, non-temporal", "channel-blocked [col/16][row][16]",
                            "contiguous 4 KB per wave chunk"};
    float us[4] = {run<0>(c), run<1>(c), run<2>(c), run<3>(c)};
    const double mb = (double)M * N * 4 / 1e6;
    for (int p = 0; p < 4; ++p) printf("%-36s %7.2f us  %7.1f GB/s\n", names[p], us[p], mb * 1e3 / us[p]);
    hipFree(c);
    return 0;
}
