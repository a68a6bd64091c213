// The C3 loss rows' HBM ceiling for their read/write mix (VERDICT r03 "what's weak" 2): 12288
// rows of V = 32128 bf16 (64,256 B), a decoder-length mask (row b·T + t valid iff t < L_b, L_b
// uniform in 1..T, ~51 % valid).  A valid row is read and written (the fused loss rows read
// the logits and write dlogits), a masked row only written with zeros (masked_row).
//   mix      one workgroup per row in row order (the product's grid)
//   mix-tail the valid rows first, then the masked rows k per workgroup (the order-list layout)
//   copy     every row read and written (the dense ceiling)
//   zero     every row only written
// Same geometry as the product's rows: 512 threads, whole 16-B vectors, nt buffer ops.
// Build: hipcc --offload-arch=gfx950 -O3 -I../trlx-t5_amd/csrc -I../include mix_probe.hip -o mix_probe
#include <stdio.h>
#include <stdlib.h>
#include "common.h"

using namespace trlx;
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int kThr = 512, kNV = 8;  // 4096 vectors >= 4016 per row

__device__ __forceinline__ void copy_row(const char* x, char* y, uint32_t bytes) {
    const __amdgpu_buffer_rsrc_t ri = make_rsrc(x, bytes), ro = make_rsrc(y, bytes);
    const int voff = threadIdx.x * 16;
    vec4u v[kNV];
#pragma unroll
    for (int k = 0; k < kNV; ++k) v[k] = __builtin_amdgcn_raw_buffer_load_b128(ri, launder_int(voff) + k * kThr * 16, 0, kAuxNT);
#pragma unroll
    for (int k = 0; k < kNV; ++k) __builtin_amdgcn_raw_buffer_store_b128(v[k], ro, launder_int(voff) + k * kThr * 16, 0, kAuxNT);
}
__device__ __forceinline__ void zero_row(char* y, uint32_t bytes) {
    const __amdgpu_buffer_rsrc_t ro = make_rsrc(y, bytes);
    const int voff = threadIdx.x * 16;
    const vec4u z = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < kNV; ++k) __builtin_amdgcn_raw_buffer_store_b128(z, ro, launder_int(voff) + k * kThr * 16, 0, kAuxNT);
}

// MODE 0 mix (row order), 1 copy, 2 zero
template <int MODE>
__global__ __launch_bounds__(kThr) void k_rows(const char* x, char* y, const int* mask, uint32_t rb) {
    const size_t off = size_t(blockIdx.x) * rb;
    if (MODE == 2 || (MODE == 0 && !mask[blockIdx.x])) {
        zero_row(y + off, rb);
        return;
    }
    copy_row(x + off, y + off, rb);
}
// valid rows first (list), then the masked rows K per workgroup
template <int K>
__global__ __launch_bounds__(kThr) void k_rows_tail(const char* x, char* y, const int* order, int nvalid, int n,
                                                    uint32_t rb) {
    const int i = blockIdx.x;
    if (i < nvalid) {
        const size_t off = size_t(order[i]) * rb;
        copy_row(x + off, y + off, rb);
        return;
    }
    for (int k = 0; k < K; ++k) {
        const int j = nvalid + (i - nvalid) * K + k;
        if (j < n) zero_row(y + size_t(order[j]) * rb, rb);
    }
}

template <typename F>
float time_it(F f, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 5; ++i) f();
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
    const int B = 256, T = 48, n = B * T;
    const uint32_t rb = 32128 * 2;
    const size_t bytes = size_t(n) * rb;
    int* hm = (int*)malloc(n * 4);
    int* ho = (int*)malloc(n * 4);
    unsigned s = 12345u;
    int nvalid = 0;
    for (int b = 0; b < B; ++b) {
        s = s * 1664525u + 1013904223u;
        const int L = 1 + int((s >> 8) % T);
        for (int t = 0; t < T; ++t) {
            hm[b * T + t] = t < L;
            nvalid += t < L;
        }
    }
    for (int i = 0, v = 0, m = nvalid; i < n; ++i) (hm[i] ? ho[v++] : ho[m++]) = i;
    char *x, *y;
    int *dm, *dord;
    CHECK(hipMalloc(&x, bytes));
    CHECK(hipMalloc(&y, bytes));
    CHECK(hipMalloc(&dm, n * 4));
    CHECK(hipMalloc(&dord, n * 4));
    CHECK(hipMemset(x, 1, bytes));
    CHECK(hipMemcpy(dm, hm, n * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dord, ho, n * 4, hipMemcpyHostToDevice));
    const double mix_bytes = double(nvalid) * 2 * rb + double(n - nvalid) * rb;
    printf("rows %d valid %d (%.3f), mix bytes %.0f\n", n, nvalid, double(nvalid) / n, mix_bytes);
    for (int rep = 0; rep < 3; ++rep) {
        float ms = time_it([&] { hipLaunchKernelGGL(k_rows<0>, dim3(n), dim3(kThr), 0, 0, x, y, dm, rb); }, 20);
        printf("mix (row order)       %7.1f us %7.1f GB/s (%.3f of 8 TB/s)\n", ms * 1e3, mix_bytes / ms / 1e6,
               mix_bytes / ms / 1e6 / 8000.0);
        const int nb4 = nvalid + (n - nvalid + 3) / 4;
        ms = time_it([&] { hipLaunchKernelGGL(k_rows_tail<4>, dim3(nb4), dim3(kThr), 0, 0, x, y, dord, nvalid, n, rb); }, 20);
        printf("mix-tail (4 zero rows/wg) %7.1f us %7.1f GB/s\n", ms * 1e3, mix_bytes / ms / 1e6);
        const int nb1 = n;
        ms = time_it([&] { hipLaunchKernelGGL(k_rows_tail<1>, dim3(nb1), dim3(kThr), 0, 0, x, y, dord, nvalid, n, rb); }, 20);
        printf("mix-tail (1 zero row/wg)  %7.1f us %7.1f GB/s\n", ms * 1e3, mix_bytes / ms / 1e6);
        ms = time_it([&] { hipLaunchKernelGGL(k_rows<1>, dim3(n), dim3(kThr), 0, 0, x, y, dm, rb); }, 20);
        printf("copy (all rows r+w)   %7.1f us %7.1f GB/s\n", ms * 1e3, 2.0 * bytes / ms / 1e6);
        ms = time_it([&] { hipLaunchKernelGGL(k_rows<2>, dim3(n), dim3(kThr), 0, 0, x, y, dm, rb); }, 20);
        printf("zero (all rows w)     %7.1f us %7.1f GB/s\n", ms * 1e3, 1.0 * bytes / ms / 1e6);
    }
    return 0;
}
