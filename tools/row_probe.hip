// Structure probe for the register-resident R+W row kernel (C2 bf16 shape, 6144 rows of
// 50257): which part of the fused loss kernel costs bandwidth?  Variants, all moving one
// read + one write of every row with 16-B nt buffer ops, 512-thread workgroups x 13 vectors:
//   0  copy only (load row -> store row), no barrier
//   1  copy + 2 block reductions (barriers) between load and store
//   2  copy + 1 block reduction
//   3  full arithmetic (max, sum-exp, dlogits = -g*exp(x - lse)), 2 reductions
//   4  full arithmetic, 1 combined (max, sum) reduction (per-thread online merge)
// Build: hipcc --offload-arch=gfx950 -O3 -I../trlx-t5_amd/csrc -I../include row_probe.hip -o row_probe
#include <stdio.h>
#include <vector>
#include "common.h"

using namespace trlx;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int NV, int VAR>
__global__ __launch_bounds__(512) void k_probe(const uint16_t* x, uint16_t* dx, int64_t V, int64_t stride) {
    __shared__ float sh_a[8], sh_b[8];
    const int tid = threadIdx.x, nthr = blockDim.x;
    const uint16_t* row = x + int64_t(blockIdx.x) * stride;
    uint16_t* drow = dx + int64_t(blockIdx.x) * stride;
    const RowSplit<BF16T> s(row, V);
    const int nvec = int(s.nvec);
    const __amdgpu_buffer_rsrc_t rin = make_rsrc(row + s.head, uint32_t(nvec) * 16u);
    const __amdgpu_buffer_rsrc_t rout = make_rsrc(drow + s.head, uint32_t(nvec) * 16u);
    const int voff = tid * 16;
    vec4u v[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k)
        v[k] = __builtin_amdgcn_raw_buffer_load_b128(rin, launder_int(voff) + k * nthr * 16, 0, kAuxNT);
    float g = 0.5f, lse = 0.0f;
    if (VAR == 1 || VAR == 2) {
        float a = 0.f;
#pragma unroll
        for (int k = 0; k < NV; ++k) a += __uint_as_float(v[k].x);
        a = block_sum(a, sh_a);
        if (VAR == 1) a = block_max(a, sh_b);
        g = a > 1e30f ? 1.f : 0.5f;
    }
    if (VAR == 3) {
        float m = -INFINITY;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            float f[8];
            BF16T::unpack(v[k], f);
            float mk = f[0];
#pragma unroll
            for (int e = 1; e < 8; ++e) mk = fmaxf(mk, f[e]);
            m = (tid + k * nthr < nvec) ? fmaxf(m, mk) : m;
        }
        m = block_max(m, sh_a);
#pragma unroll
        for (int k = 0; k < NV; ++k) launder(v[k]);
        const float ml2e = -m * kLog2e;
        float sum = 0.f;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            float f[8];
            BF16T::unpack(v[k], f);
            float sk = 0.0f;
#pragma unroll
            for (int e = 0; e < 8; ++e) sk += exp2_fast(fmaf(f[e], kLog2e, ml2e));
            sum += (tid + k * nthr < nvec) ? sk : 0.0f;
        }
        sum = block_sum(sum, sh_b);
#pragma unroll
        for (int k = 0; k < NV; ++k) launder(v[k]);
        lse = m + logf(sum);
    }
    if (VAR == 4) {
        float m = -INFINITY;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            float f[8];
            BF16T::unpack(v[k], f);
            float mk = f[0];
#pragma unroll
            for (int e = 1; e < 8; ++e) mk = fmaxf(mk, f[e]);
            m = (tid + k * nthr < nvec) ? fmaxf(m, mk) : m;
        }
#pragma unroll
        for (int k = 0; k < NV; ++k) launder(v[k]);
        const float ml2e = -m * kLog2e;
        float sum = 0.f;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            float f[8];
            BF16T::unpack(v[k], f);
            float sk = 0.0f;
#pragma unroll
            for (int e = 0; e < 8; ++e) sk += exp2_fast(fmaf(f[e], kLog2e, ml2e));
            sum += (tid + k * nthr < nvec) ? sk : 0.0f;
        }
#pragma unroll
        for (int k = 0; k < NV; ++k) launder(v[k]);
        // wave merge of (m, sum) then one LDS exchange
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const float m2 = __shfl_xor(m, off, kWave), s2 = __shfl_xor(sum, off, kWave);
            const float nm = fmaxf(m, m2);
            sum = (m == -INFINITY ? 0.f : sum * exp2_fast((m - nm) * kLog2e)) +
                  (m2 == -INFINITY ? 0.f : s2 * exp2_fast((m2 - nm) * kLog2e));
            m = nm;
        }
        if ((tid & 63) == 0) { sh_a[tid / 64] = m; sh_b[tid / 64] = sum; }
        __syncthreads();
        float M = sh_a[0];
        for (int w = 1; w < nthr / 64; ++w) M = fmaxf(M, sh_a[w]);
        float S = 0.f;
        for (int w = 0; w < nthr / 64; ++w) S += sh_b[w] * exp2_fast((sh_a[w] - M) * kLog2e);
        lse = M + logf(S);
    }
    const float lse_l2e = -lse * kLog2e;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        vec4u o = v[k];
        if (VAR >= 3) {
            float f[8];
            BF16T::unpack(v[k], f);
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] = -g * exp2_fast(fmaf(f[e], kLog2e, lse_l2e));
            o = BF16T::pack(f);
        } else if (g == 1.f) {
            o.x += 1u;
        }
        __builtin_amdgcn_raw_buffer_store_b128(o, rout, launder_int(voff) + k * nthr * 16, 0, kAuxNT);
    }
}

template <typename F>
float time_it(F f, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    f();
    f();
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int i = 0; i < reps; ++i) f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main() {
    const int64_t rows = 128 * 48, V = 50257;
    const size_t bytes = size_t(rows) * V * 2;
    uint16_t *x, *dx;
    CHECK(hipMalloc(&x, bytes + 64));
    CHECK(hipMalloc(&dx, bytes + 64));
    std::vector<uint16_t> h(V);
    for (int64_t j = 0; j < V; ++j) h[j] = 0x3f80 + uint16_t(j % 64);  // bf16 1.0 .. ~1.5
    for (int64_t r = 0; r < rows; ++r) CHECK(hipMemcpy(x + r * V, h.data(), V * 2, hipMemcpyHostToDevice));
    const char* names[] = {"copy", "copy+2 barriers", "copy+1 barrier", "full arith 2 reductions",
                           "full arith 1 reduction"};
    for (int rep = 0; rep < 2; ++rep)
        for (int var = 0; var < 5; ++var) {
            float ms = time_it([&] {
                switch (var) {
                    case 0: hipLaunchKernelGGL((k_probe<13, 0>), dim3(rows), dim3(512), 0, 0, x, dx, V, V); break;
                    case 1: hipLaunchKernelGGL((k_probe<13, 1>), dim3(rows), dim3(512), 0, 0, x, dx, V, V); break;
                    case 2: hipLaunchKernelGGL((k_probe<13, 2>), dim3(rows), dim3(512), 0, 0, x, dx, V, V); break;
                    case 3: hipLaunchKernelGGL((k_probe<13, 3>), dim3(rows), dim3(512), 0, 0, x, dx, V, V); break;
                    case 4: hipLaunchKernelGGL((k_probe<13, 4>), dim3(rows), dim3(512), 0, 0, x, dx, V, V); break;
                }
            }, 10);
            printf("%-26s %8.1f us  %7.1f GB/s (R+W)\n", names[var], ms * 1e3, 2.0 * bytes / ms / 1e6);
        }
    return 0;
}
