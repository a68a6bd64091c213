// Long fp32 rows (V = 50257: 201,024 B), read into VGPRs, a block-wide max, written back
// scaled: the R+W shape of the ILQL / fp32 PPO loss rows at two rows in flight per CU.
// Question: does a row workgroup's dispatch + load-latency bubble cost bandwidth, and does a
// persistent workgroup that loads row i+1 into the registers row i's stores just released
// (interleaved per vector step) recover it?
//   rowwg        one workgroup per row (the product's structure)
//   persist      512 persistent workgroups, row i+1 loaded after row i's stores
//   persist-il   512 persistent workgroups, load of row i+1 step k right after store of row i step k
// Build: hipcc --offload-arch=gfx950 -O3 -I../trlx-t5_amd/csrc -I../include rowpipe_probe.hip -o rowpipe_probe
#include <stdio.h>
#include "common.h"

using namespace trlx;
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int THR = 512, NV = 25;
constexpr uint32_t kRowBytes = 201024;     // 12,564 16-B vectors
constexpr int64_t kRowStride = 201216;     // 256-B multiple

__device__ __forceinline__ float probe_block_max(float m, float* sh) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = m;
    __syncthreads();
    float r = sh[0];
#pragma unroll
    for (int w = 1; w < THR / 64; ++w) r = fmaxf(r, sh[w]);
    return r;
}

template <int SPOL>
__device__ __forceinline__ void st(const vec4u& v, float s, __amdgpu_buffer_rsrc_t r, int off) {
    vec4u o;
    o.x = __float_as_uint(__uint_as_float(v.x) * s);
    o.y = __float_as_uint(__uint_as_float(v.y) * s);
    o.z = __float_as_uint(__uint_as_float(v.z) * s);
    o.w = __float_as_uint(__uint_as_float(v.w) * s);
    store_grad_b128(o, r, off, SPOL);
}

__device__ __forceinline__ float vmax(const vec4u* v) {
    float m = -INFINITY;
#pragma unroll
    for (int k = 0; k < NV; ++k)
        m = fmaxf(m, fmaxf(fmaxf(__uint_as_float(v[k].x), __uint_as_float(v[k].y)),
                           fmaxf(__uint_as_float(v[k].z), __uint_as_float(v[k].w))));
    return m;
}

template <int SPOL, int LAUX = kAuxNT>
__global__ __launch_bounds__(THR, 4) void k_rowwg(const char* x, char* y, int R) {
    __shared__ float sh[THR / 64];
    const int64_t r = blockIdx.x;
    const __amdgpu_buffer_rsrc_t ri = make_rsrc(x + r * kRowStride, kRowBytes);
    const __amdgpu_buffer_rsrc_t ro = make_rsrc(y + r * kRowStride, kRowBytes);
    const int voff = threadIdx.x * 16;
    vec4u v[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = __builtin_amdgcn_raw_buffer_load_b128(ri, launder_int(voff) + k * THR * 16, 0, LAUX);
    const float s = 1.0f / (1.0f + fabsf(probe_block_max(vmax(v), sh)));
#pragma unroll
    for (int k = 0; k < NV; ++k) st<SPOL>(v[k], s, ro, launder_int(voff) + k * THR * 16);
}

template <int SPOL, bool IL>
__global__ __launch_bounds__(THR, 4) void k_persist(const char* x, char* y, int R) {
    __shared__ float sh[THR / 64];
    const int voff = threadIdx.x * 16;
    int64_t r = blockIdx.x;
    vec4u v[NV];
    {
        const __amdgpu_buffer_rsrc_t ri = make_rsrc(x + r * kRowStride, kRowBytes);
#pragma unroll
        for (int k = 0; k < NV; ++k) v[k] = __builtin_amdgcn_raw_buffer_load_b128(ri, launder_int(voff) + k * THR * 16, 0, kAuxNT);
    }
    while (r < R) {  // every workgroup leaves once its rows are done
        const float s = 1.0f / (1.0f + fabsf(probe_block_max(vmax(v), sh)));
        const __amdgpu_buffer_rsrc_t ro = make_rsrc(y + r * kRowStride, kRowBytes);
        const int64_t rn = r + gridDim.x;
        const __amdgpu_buffer_rsrc_t rn_i = make_rsrc(x + (rn < R ? rn : r) * kRowStride, rn < R ? kRowBytes : 0u);
        if (IL) {
#pragma unroll
            for (int k = 0; k < NV; ++k) {
                st<SPOL>(v[k], s, ro, launder_int(voff) + k * THR * 16);
                v[k] = __builtin_amdgcn_raw_buffer_load_b128(rn_i, launder_int(voff) + k * THR * 16, 0, kAuxNT);
            }
        } else {
#pragma unroll
            for (int k = 0; k < NV; ++k) st<SPOL>(v[k], s, ro, launder_int(voff) + k * THR * 16);
#pragma unroll
            for (int k = 0; k < NV; ++k) v[k] = __builtin_amdgcn_raw_buffer_load_b128(rn_i, launder_int(voff) + k * THR * 16, 0, kAuxNT);
        }
        r = rn;
    }
}

template <class K>
static float timeit(K launch, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    launch();
    hipDeviceSynchronize();
    float best = 1e30f, tot = 0.0f;
    for (int i = 0; i < reps; ++i) {
        hipEventRecord(a, 0);
        launch();
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        tot += ms;
        best = ms < best ? ms : best;
    }
    return tot / reps;
}

int main() {
    const int R = 24320;
    char *x, *y;
    CHECK(hipMalloc(&x, size_t(R) * kRowStride));
    CHECK(hipMalloc(&y, size_t(R) * kRowStride));
    CHECK(hipMemset(x, 0x3c, size_t(R) * kRowStride));
    const double bytes = 2.0 * R * double(kRowBytes);
    const int G = 512;
    struct V { const char* name; float ms; } res[12];
    int n = 0;
    for (int pass = 0; pass < 2; ++pass) {
        n = 0;
        res[n++] = {"rowwg nt", timeit([&] { hipLaunchKernelGGL((k_rowwg<kStoreNT>), dim3(R), dim3(THR), 0, 0, x, y, R); }, 10)};
        res[n++] = {"rowwg sc1", timeit([&] { hipLaunchKernelGGL((k_rowwg<kStoreSC1>), dim3(R), dim3(THR), 0, 0, x, y, R); }, 10)};
        res[n++] = {"rowwg none", timeit([&] { hipLaunchKernelGGL((k_rowwg<kStoreNone>), dim3(R), dim3(THR), 0, 0, x, y, R); }, 10)};
        res[n++] = {"rowwg nt ld-default", timeit([&] { hipLaunchKernelGGL((k_rowwg<kStoreNT, 0>), dim3(R), dim3(THR), 0, 0, x, y, R); }, 10)};
        res[n++] = {"rowwg ntsc1", timeit([&] { hipLaunchKernelGGL((k_rowwg<kStoreNTSC1>), dim3(R), dim3(THR), 0, 0, x, y, R); }, 10)};
        res[n++] = {"persist nt", timeit([&] { hipLaunchKernelGGL((k_persist<kStoreNT, false>), dim3(G), dim3(THR), 0, 0, x, y, R); }, 10)};
        res[n++] = {"persist-il nt", timeit([&] { hipLaunchKernelGGL((k_persist<kStoreNT, true>), dim3(G), dim3(THR), 0, 0, x, y, R); }, 10)};
        res[n++] = {"persist-il sc1", timeit([&] { hipLaunchKernelGGL((k_persist<kStoreSC1, true>), dim3(G), dim3(THR), 0, 0, x, y, R); }, 10)};
        res[n++] = {"persist-il nt G768", timeit([&] { hipLaunchKernelGGL((k_persist<kStoreNT, true>), dim3(768), dim3(THR), 0, 0, x, y, R); }, 10)};
    }
    CHECK(hipGetLastError());
    for (int i = 0; i < n; ++i) printf("%-20s %8.1f us  %6.3f TB/s\n", res[i].name, res[i].ms * 1e3, bytes / (res[i].ms * 1e-3) / 1e12);
    return 0;
}
