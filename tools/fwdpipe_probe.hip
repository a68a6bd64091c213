// Structure probe for the read-only experience rows (C2: 12288 bf16 rows of 50257, the policy
// and reference rows of 6144 tokens): does a persistent workgroup that loads row i+1 while it
// reduces row i beat one row per workgroup?  Both do the product kernel's arithmetic per row
// (raw-bits bf16 max by v_pk_max_i16, one block max, packed-fp32 exp-sum, one block sum, one
// fp32 store per row) on 16-B nt buffer loads with the 256-B line shift.
//   variant 0  one row per 512-thread workgroup, 13 vectors per thread (the product layout)
//   variant 1  persistent 512-thread workgroups, two 13-vector register sets: row i+1's loads
//              are issued before row i's reductions (grid = G workgroups, rows strided by G)
// Build: hipcc --offload-arch=gfx950 -O3 -I../trlx-t5_amd/csrc -I../include fwdpipe_probe.hip -o fwdpipe_probe
#include <stdio.h>
#include <vector>
#include "common.h"

using namespace trlx;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int NV = 13;

__device__ __forceinline__ void load_row(const uint16_t* row, int V, vec4u (&v)[NV], int& nvec, int& vbase) {
    const RowSplit<BF16T> s(row, V);
    nvec = int(s.nvec);
    const __amdgpu_buffer_rsrc_t rin = make_rsrc(row + s.head, uint32_t(nvec) * 16u);
    const int shift = line_shift(row + s.head);
    vbase = int(threadIdx.x) - shift;
    const int voff = vbase * 16;
#pragma unroll
    for (int k = 0; k < NV; ++k)
        v[k] = __builtin_amdgcn_raw_buffer_load_b128(rin, launder_int(voff) + k * 512 * 16, 0, kAuxNT);
}

__device__ __forceinline__ float reduce_row(vec4u (&v)[NV], int nvec, int vbase, float* sh_m, float* sh_s) {
    constexpr uint32_t kNeg0 = 0x80008000u;
    uint32_t acc = kNeg0;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const uint32_t p = pk_max_i16(pk_max_i16(v[k].x, v[k].y), pk_max_i16(v[k].z, v[k].w));
        acc = pk_max_i16(acc, unsigned(vbase + k * 512) < unsigned(nvec) ? p : kNeg0);
    }
    const int mi = max(int(int16_t(acc & 0xffffu)), int(acc) >> 16);
    const float m = block_max(__uint_as_float(uint32_t(mi) << 16), sh_m);
#pragma unroll
    for (int k = 0; k < NV; ++k) launder(v[k]);
    const float ml2e = -m * kLog2e;
    const f32x2 l2e2 = f2_splat(kLog2e), ml2e2 = f2_splat(ml2e), zero2 = f2_splat(0.0f);
    f32x2 s2 = zero2;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        float f[8];
        BF16T::unpack(v[k], f);
        const f32x2 sk = exp_pair_sum(f, l2e2, ml2e2);
        s2 += (unsigned(vbase + k * 512) < unsigned(nvec)) ? sk : zero2;
    }
    const float sum = block_sum(s2.x + s2.y, sh_s);
    return m + logf(sum);
}

__global__ __launch_bounds__(512) void k_row(const uint16_t* x, float* out, int V, int64_t stride, int R) {
    __shared__ float sh_m[8], sh_s[8];
    vec4u v[NV];
    int nvec, vbase;
    load_row(x + int64_t(blockIdx.x) * stride, V, v, nvec, vbase);
    const float lse = reduce_row(v, nvec, vbase, sh_m, sh_s);
    if (threadIdx.x == 0) out[blockIdx.x] = lse;
}

__global__ __launch_bounds__(512, 2) void k_persist(const uint16_t* x, float* out, int V, int64_t stride, int R) {
    __shared__ float sh_m[2][8], sh_s[2][8];
    vec4u a[NV], b[NV];
    int na, ba, nb, bb;
    int r = blockIdx.x;
    if (r >= R) return;
    load_row(x + int64_t(r) * stride, V, a, na, ba);
    for (;;) {  // two rows per iteration, the register sets in fixed roles
        const int r1 = r + int(gridDim.x);
        if (r1 < R) load_row(x + int64_t(r1) * stride, V, b, nb, bb);
        const float l0 = reduce_row(a, na, ba, sh_m[0], sh_s[0]);
        if (threadIdx.x == 0) out[r] = l0;
        if (r1 >= R) break;
        const int r2 = r1 + int(gridDim.x);
        if (r2 < R) load_row(x + int64_t(r2) * stride, V, a, na, ba);
        const float l1 = reduce_row(b, nb, bb, sh_m[1], sh_s[1]);
        if (threadIdx.x == 0) out[r1] = l1;
        if (r2 >= R) break;
        r = r2;
    }
}

int main() {
    const int V = 50257, R = 12288;
    const int64_t stride = V;
    const size_t bytes = size_t(R) * stride * 2;
    uint16_t* x;
    float* out;
    CHECK(hipMalloc(&x, bytes));
    CHECK(hipMalloc(&out, R * 4));
    std::vector<uint16_t> h(size_t(R) * stride);
    for (size_t i = 0; i < h.size(); ++i) h[i] = uint16_t(0x3f80 + (i * 2654435761u >> 24) % 64);
    CHECK(hipMemcpy(x, h.data(), bytes, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const double gb = double(R) * V * 2 / 1e9;
    for (int round = 0; round < 3; ++round) {
        for (int var = 0; var < 4; ++var) {
            const int grid = var == 0 ? R : (var == 1 ? 512 : (var == 2 ? 768 : 1024));
            for (int it = 0; it < 40; ++it) {  // warm
                if (var == 0) hipLaunchKernelGGL(k_row, dim3(grid), dim3(512), 0, 0, x, out, V, stride, R);
                else hipLaunchKernelGGL(k_persist, dim3(grid), dim3(512), 0, 0, x, out, V, stride, R);
            }
            CHECK(hipEventRecord(e0, 0));
            const int iters = 100;
            for (int it = 0; it < iters; ++it) {
                if (var == 0) hipLaunchKernelGGL(k_row, dim3(grid), dim3(512), 0, 0, x, out, V, stride, R);
                else hipLaunchKernelGGL(k_persist, dim3(grid), dim3(512), 0, 0, x, out, V, stride, R);
            }
            CHECK(hipEventRecord(e1, 0));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1e3 / iters;
            printf("round %d %s grid %5d: %8.2f us/launch  %.3f TB/s\n", round,
                   var == 0 ? "one-row    " : "persist-2buf", grid, us, gb / us * 1e3);
        }
    }
    return 0;
}
