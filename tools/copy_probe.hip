// R+W copy structure sweep: one workgroup copies one contiguous chunk of THR x NV 16-B
// vectors (all NV loads in flight, then NV stores), nt buffer ops, 1.24 GB moved.  Tells
// which per-workgroup footprint the HBM sustains best for read-then-write rows.
// Build: hipcc --offload-arch=gfx950 -O3 -I../trlx-t5_amd/csrc -I../include copy_probe.hip -o copy_probe
#include <stdio.h>
#include "common.h"

using namespace trlx;
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int THR, int NV, int WAVES>
__global__ __launch_bounds__(THR, WAVES) void k_copy(const char* x, char* y, uint32_t chunk) {
    const char* src = x + size_t(blockIdx.x) * chunk;
    char* dst = y + size_t(blockIdx.x) * chunk;
    const __amdgpu_buffer_rsrc_t ri = make_rsrc(src, chunk), ro = make_rsrc(dst, chunk);
    const int voff = threadIdx.x * 16;
    vec4u v[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = __builtin_amdgcn_raw_buffer_load_b128(ri, launder_int(voff) + k * THR * 16, 0, kAuxNT);
#pragma unroll
    for (int k = 0; k < NV; ++k) __builtin_amdgcn_raw_buffer_store_b128(v[k], ro, launder_int(voff) + k * THR * 16, 0, kAuxNT);
}

// wave-major: wave w copies the contiguous vectors [w*NV*64, (w+1)*NV*64) of the row
template <int ALIGN, int NV, int THR>
__global__ __launch_bounds__(THR) void k_rowcopy_wm(const uint16_t* x, uint16_t* y, int64_t V) {
    const uint16_t* row = x + int64_t(blockIdx.x) * V;
    uint16_t* drow = y + int64_t(blockIdx.x) * V;
    const uintptr_t a = reinterpret_cast<uintptr_t>(row);
    const int head = int(((ALIGN - (a % ALIGN)) % ALIGN) / 2);
    const int nvec = int((V - head) / 8);
    const __amdgpu_buffer_rsrc_t ri = make_rsrc(row + head, uint32_t(nvec) * 16u);
    const __amdgpu_buffer_rsrc_t ro = make_rsrc(drow + head, uint32_t(nvec) * 16u);
    if (threadIdx.x < head) drow[threadIdx.x] = row[threadIdx.x];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int voff = (w * NV * 64 + lane) * 16;
    vec4u v[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = __builtin_amdgcn_raw_buffer_load_b128(ri, launder_int(voff) + k * 64 * 16, 0, kAuxNT);
#pragma unroll
    for (int k = 0; k < NV; ++k) __builtin_amdgcn_raw_buffer_store_b128(v[k], ro, launder_int(voff) + k * 64 * 16, 0, kAuxNT);
}

// read-only row kernel (like the experience forward): k-major vs wave-major, xor-reduce
template <int ALIGN, int NV, int THR, bool WM>
__global__ __launch_bounds__(THR) void k_rowread(const uint16_t* x, int64_t V, uint32_t* sink) {
    const uint16_t* row = x + int64_t(blockIdx.x) * V;
    const uintptr_t a = reinterpret_cast<uintptr_t>(row);
    const int head = int(((ALIGN - (a % ALIGN)) % ALIGN) / 2);
    const int nvec = int((V - head) / 8);
    const __amdgpu_buffer_rsrc_t ri = make_rsrc(row + head, uint32_t(nvec) * 16u);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int voff = WM ? (w * NV * 64 + lane) * 16 : threadIdx.x * 16;
    const int step = WM ? 64 * 16 : THR * 16;
    vec4u v[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = __builtin_amdgcn_raw_buffer_load_b128(ri, launder_int(voff) + k * step, 0, kAuxNT);
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < NV; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    if (acc == 0x12345u) sink[0] = acc;
}

template <typename F>
float time_it(F f, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    f(); f();
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int i = 0; i < reps; ++i) f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

template <int THR, int NV, int WAVES>
void run(const char* x, char* y, size_t bytes, int lds_kb = 0) {
    const uint32_t chunk = THR * NV * 16;
    const unsigned grid = unsigned(bytes / chunk);
    if (lds_kb) hipFuncSetAttribute((const void*)k_copy<THR, NV, WAVES>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_kb * 1024);
    float ms = time_it([&] { hipLaunchKernelGGL((k_copy<THR, NV, WAVES>), dim3(grid), dim3(THR), lds_kb * 1024, 0, x, y, chunk); }, 10);
    printf("thr %4d nv %2d wavesEU %d lds %3d KB chunk %7u B: %7.1f us %7.1f GB/s\n", THR, NV, WAVES, lds_kb, chunk, ms * 1e3,
           2.0 * grid * chunk / ms / 1e6);
}

// row-shaped: chunk = one 100,514-B row (stride not a multiple of 16), head-peeled body
template <int ALIGN>
__global__ __launch_bounds__(512) void k_rowcopy(const uint16_t* x, uint16_t* y, int64_t V) {
    const uint16_t* row = x + int64_t(blockIdx.x) * V;
    uint16_t* drow = y + int64_t(blockIdx.x) * V;
    const uintptr_t a = reinterpret_cast<uintptr_t>(row);
    const int head = int(((ALIGN - (a % ALIGN)) % ALIGN) / 2);
    const int nvec = int((V - head) / 8);
    const __amdgpu_buffer_rsrc_t ri = make_rsrc(row + head, uint32_t(nvec) * 16u);
    const __amdgpu_buffer_rsrc_t ro = make_rsrc(drow + head, uint32_t(nvec) * 16u);
    if (threadIdx.x < head) drow[threadIdx.x] = row[threadIdx.x];
    const int voff = threadIdx.x * 16;
    vec4u v[13];
#pragma unroll
    for (int k = 0; k < 13; ++k) v[k] = __builtin_amdgcn_raw_buffer_load_b128(ri, launder_int(voff) + k * 512 * 16, 0, kAuxNT);
#pragma unroll
    for (int k = 0; k < 13; ++k) __builtin_amdgcn_raw_buffer_store_b128(v[k], ro, launder_int(voff) + k * 512 * 16, 0, kAuxNT);
}

int main() {
    const size_t bytes = size_t(6144) * 50257 * 2;
    char *x, *y;
    CHECK(hipMalloc(&x, bytes + 4096));
    CHECK(hipMalloc(&y, bytes + 4096));
    CHECK(hipMemset(x, 1, bytes));
    CHECK(hipMemset(y, 0, bytes));
    for (int rep = 0; rep < 1; ++rep) {
        {
            float ms = time_it([&] { hipLaunchKernelGGL(k_rowcopy<16>, dim3(6144), dim3(512), 0, 0, (const uint16_t*)x, (uint16_t*)y, 50257); }, 10);
            printf("row-shaped 512x13 body 16B-aligned : %7.1f us %7.1f GB/s\n", ms * 1e3, 2.0 * bytes / ms / 1e6);
            ms = time_it([&] { hipLaunchKernelGGL(k_rowcopy<128>, dim3(6144), dim3(512), 0, 0, (const uint16_t*)x, (uint16_t*)y, 50257); }, 10);
            printf("row-shaped 512x13 body 128B-aligned: %7.1f us %7.1f GB/s\n", ms * 1e3, 2.0 * bytes / ms / 1e6);
            ms = time_it([&] { hipLaunchKernelGGL(k_rowcopy<256>, dim3(6144), dim3(512), 0, 0, (const uint16_t*)x, (uint16_t*)y, 50257); }, 10);
            printf("row-shaped 512x13 body 256B-aligned: %7.1f us %7.1f GB/s\n", ms * 1e3, 2.0 * bytes / ms / 1e6);
            ms = time_it([&] { hipLaunchKernelGGL((k_rowcopy_wm<256, 13, 512>), dim3(6144), dim3(512), 0, 0, (const uint16_t*)x, (uint16_t*)y, 50257); }, 10);
            printf("row-shaped 512x13 wave-major 256B  : %7.1f us %7.1f GB/s\n", ms * 1e3, 2.0 * bytes / ms / 1e6);
            ms = time_it([&] { hipLaunchKernelGGL((k_rowcopy_wm<256, 7, 1024>), dim3(6144), dim3(1024), 0, 0, (const uint16_t*)x, (uint16_t*)y, 50257); }, 10);
            printf("row-shaped 1024x7 wave-major 256B  : %7.1f us %7.1f GB/s\n", ms * 1e3, 2.0 * bytes / ms / 1e6);
            ms = time_it([&] { hipLaunchKernelGGL((k_rowcopy_wm<256, 25, 256>), dim3(6144), dim3(256), 0, 0, (const uint16_t*)x, (uint16_t*)y, 50257); }, 10);
            printf("row-shaped 256x25 wave-major 256B  : %7.1f us %7.1f GB/s\n", ms * 1e3, 2.0 * bytes / ms / 1e6);
            uint32_t* sink = (uint32_t*)y;
            ms = time_it([&] { hipLaunchKernelGGL((k_rowread<256, 13, 512, false>), dim3(6144), dim3(512), 0, 0, (const uint16_t*)x, 50257, sink); }, 10);
            printf("read rows 512x13 k-major           : %7.1f us %7.1f GB/s\n", ms * 1e3, 1.0 * bytes / ms / 1e6);
            ms = time_it([&] { hipLaunchKernelGGL((k_rowread<256, 13, 512, true>), dim3(6144), dim3(512), 0, 0, (const uint16_t*)x, 50257, sink); }, 10);
            printf("read rows 512x13 wave-major        : %7.1f us %7.1f GB/s\n", ms * 1e3, 1.0 * bytes / ms / 1e6);
            ms = time_it([&] { hipLaunchKernelGGL((k_rowread<256, 7, 1024, false>), dim3(6144), dim3(1024), 0, 0, (const uint16_t*)x, 50257, sink); }, 10);
            printf("read rows 1024x7 k-major           : %7.1f us %7.1f GB/s\n", ms * 1e3, 1.0 * bytes / ms / 1e6);
            ms = time_it([&] { hipLaunchKernelGGL((k_rowread<256, 25, 256, false>), dim3(6144), dim3(256), 0, 0, (const uint16_t*)x, 50257, sink); }, 10);
            printf("read rows 256x25 k-major           : %7.1f us %7.1f GB/s\n", ms * 1e3, 1.0 * bytes / ms / 1e6);
        }
        run<256, 4, 1>(x, y, bytes);
        run<256, 8, 1>(x, y, bytes);
        run<256, 13, 1>(x, y, bytes);
        run<256, 26, 1>(x, y, bytes);
        run<512, 4, 1>(x, y, bytes);
        run<512, 7, 1>(x, y, bytes);
        run<512, 13, 1>(x, y, bytes);
        run<512, 13, 6>(x, y, bytes);
        run<1024, 4, 1>(x, y, bytes);
        run<1024, 7, 1>(x, y, bytes);
        run<1024, 13, 1>(x, y, bytes);
        run<128, 13, 1>(x, y, bytes);
        run<64, 13, 1>(x, y, bytes);
        run<128, 4, 1>(x, y, bytes);
        run<64, 4, 1>(x, y, bytes);
        run<64, 1, 1>(x, y, bytes);
    }
    return 0;
}
