// HBM ceiling probe for MI355X: read-only and read+write streams of a large buffer with
// 16-B vectors, per cache policy and grid shape.  Gives the measured ceilings the row
// kernels are compared against.  Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int AUXL>
__global__ void k_read(const v4u* __restrict__ in, size_t n, uint32_t* out) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)in, 0, 0x7fffffff, 0x00020000);
    (void)r;
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
        v4u v;
        if (AUXL == 2) v = __builtin_nontemporal_load(in + i);
        else v = in[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int AUXL, int AUXS, int U>
__global__ void k_copy(const v4u* __restrict__ in, v4u* __restrict__ out, size_t n) {
    const size_t stride = size_t(gridDim.x) * blockDim.x;
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += stride * U) {
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t j = i + u * stride;
            if (j < n) v[u] = AUXL == 2 ? __builtin_nontemporal_load(in + j) : in[j];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t j = i + u * stride;
            if (j < n) {
                v4u w = v[u] + 1u;
                if (AUXS == 2) __builtin_nontemporal_store(w, out + j);
                else if (AUXS == 16) __hip_atomic_store((unsigned long long*)(out + j), (unsigned long long)w.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else out[j] = w;
            }
        }
    }
}

// One block copies one contiguous chunk of blockDim*U vectors (the row kernels' pattern).
template <int AUX, int U>
__global__ void k_copy_chunk(const v4u* __restrict__ in, v4u* __restrict__ out, size_t n) {
    const size_t base = size_t(blockIdx.x) * blockDim.x * U + threadIdx.x;
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t j = base + size_t(u) * blockDim.x;
        if (j < n) v[u] = AUX ? __builtin_nontemporal_load(in + j) : in[j];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t j = base + size_t(u) * blockDim.x;
        if (j < n) {
            if (AUX) __builtin_nontemporal_store(v[u] + 1u, out + j);
            else out[j] = v[u] + 1u;
        }
    }
}

template <typename F>
float time_it(F f, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
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
    const size_t bytes = size_t(618) << 20;  // ~ one C2 bf16 logits tensor
    const size_t n = bytes / 16;
    v4u *in, *out;
    uint32_t* sink;
    CHECK(hipMalloc(&in, bytes));
    CHECK(hipMalloc(&out, bytes));
    CHECK(hipMalloc(&sink, 16));
    CHECK(hipMemset(in, 1, bytes));
    CHECK(hipMemset(out, 0, bytes));
    const int grids[] = {1024, 2048, 4096, 8192};
    for (int g : grids) {
        float ms = time_it([&] { hipLaunchKernelGGL((k_read<0>), dim3(g), dim3(256), 0, 0, in, n, sink); }, 10);
        float ms2 = time_it([&] { hipLaunchKernelGGL((k_read<2>), dim3(g), dim3(256), 0, 0, in, n, sink); }, 10);
        printf("read   grid %5d x256: plain %7.1f GB/s  nt %7.1f GB/s\n", g, bytes / ms / 1e6, bytes / ms2 / 1e6);
    }
    for (int g : grids) {
        float a = time_it([&] { hipLaunchKernelGGL((k_copy<0, 0, 4>), dim3(g), dim3(256), 0, 0, in, out, n); }, 10);
        float b = time_it([&] { hipLaunchKernelGGL((k_copy<2, 2, 4>), dim3(g), dim3(256), 0, 0, in, out, n); }, 10);
        float c = time_it([&] { hipLaunchKernelGGL((k_copy<2, 0, 4>), dim3(g), dim3(256), 0, 0, in, out, n); }, 10);
        float d = time_it([&] { hipLaunchKernelGGL((k_copy<0, 2, 4>), dim3(g), dim3(256), 0, 0, in, out, n); }, 10);
        printf("copy   grid %5d x256 (R+W GB/s): ld/st plain %7.1f  nt/nt %7.1f  nt/plain %7.1f  plain/nt %7.1f\n", g,
               2 * bytes / a / 1e6, 2 * bytes / b / 1e6, 2 * bytes / c / 1e6, 2 * bytes / d / 1e6);
    }
    for (int thr : {256, 512, 1024}) {
        for (int aux : {0, 1}) {
            float a = time_it([&] {
                const unsigned g4 = unsigned((n + thr * 4 - 1) / (thr * 4));
                const unsigned g8 = unsigned((n + thr * 8 - 1) / (thr * 8));
                const unsigned g16 = unsigned((n + thr * 16 - 1) / (thr * 16));
                (void)g8; (void)g16;
                if (aux) hipLaunchKernelGGL((k_copy_chunk<1, 4>), dim3(g4), dim3(thr), 0, 0, in, out, n);
                else hipLaunchKernelGGL((k_copy_chunk<0, 4>), dim3(g4), dim3(thr), 0, 0, in, out, n);
            }, 10);
            float b = time_it([&] {
                const unsigned g8 = unsigned((n + thr * 8 - 1) / (thr * 8));
                if (aux) hipLaunchKernelGGL((k_copy_chunk<1, 8>), dim3(g8), dim3(thr), 0, 0, in, out, n);
                else hipLaunchKernelGGL((k_copy_chunk<0, 8>), dim3(g8), dim3(thr), 0, 0, in, out, n);
            }, 10);
            float c = time_it([&] {
                const unsigned g16 = unsigned((n + thr * 16 - 1) / (thr * 16));
                if (aux) hipLaunchKernelGGL((k_copy_chunk<1, 16>), dim3(g16), dim3(thr), 0, 0, in, out, n);
                else hipLaunchKernelGGL((k_copy_chunk<0, 16>), dim3(g16), dim3(thr), 0, 0, in, out, n);
            }, 10);
            printf("chunk  %4d thr %s (R+W GB/s): U4 %7.1f  U8 %7.1f  U16 %7.1f\n", thr, aux ? "nt   " : "plain",
                   2 * bytes / a / 1e6, 2 * bytes / b / 1e6, 2 * bytes / c / 1e6);
        }
    }
    hipFree(in);
    hipFree(out);
    hipFree(sink);
    return 0;
}
