// Cost of cross-stream ordering points on MI355X (ROCm 7): a chain of short kernels on a
// "main" stream, with per-iteration variants of how a side stream is ordered after / joined
// back into it.  Prints us/iteration for each variant (median of 5 repetitions).
//   none         k; k                                   (baseline)
//   record       k; record(ev); k                        (marker on main)
//   stopev       k(stop=ev); k                           (event on the kernel's dispatch)
//   rec+sidewait k; record(ev); side waits ev; k         (side stream ordered after main)
//   stop+sidewait
//   join         side: record(ev2) early; main: k; wait(ev2); k   (satisfied join on main)
//   full         k(stop=ev); side waits ev, side k2, record ev2; k; main waits ev2; k
// Build: hipcc --offload-arch=gfx950 -O2 tools/join_probe.hip -o tools/join_probe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
            return 1;                                                                             \
        }                                                                                         \
    } while (0)

__global__ void k_spin(float* p, int n) {  // ~5-10 us of work on a few blocks
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    float v = p[i];
    for (int r = 0; r < n; ++r) v = v * 0.999f + 0.001f;
    p[i] = v;
}

int main() {
    float* buf;
    CK(hipMalloc(&buf, 1 << 20));
    CK(hipMemset(buf, 0, 1 << 20));
    hipStream_t s, side;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
    const unsigned flags[2] = {hipEventDisableTiming | 0x20000000u, hipEventDisableTiming};
    const char* fname[2] = {"nofence", "default"};
    const int iters = 2000, spin = 2000;
    for (int fi = 0; fi < 2; ++fi) {
        std::vector<hipEvent_t> ev(8), ev2(8);
        for (int i = 0; i < 8; ++i) {
            CK(hipEventCreateWithFlags(&ev[i], flags[fi]));
            CK(hipEventCreateWithFlags(&ev2[i], flags[fi]));
        }
        const char* names[] = {"none", "record", "stopev", "rec+sidewait", "stop+sidewait", "join", "full"};
        for (int v = 0; v < 7; ++v) {
            std::vector<double> reps;
            for (int rep = 0; rep < 5; ++rep) {
                CK(hipDeviceSynchronize());
                auto t0 = std::chrono::steady_clock::now();
                for (int it = 0; it < iters; ++it) {
                    hipEvent_t e = ev[it & 7], e2 = ev2[it & 7];
                    if (v == 5) {
                        CK(hipEventRecord(e2, side));
                    }
                    if (v == 2 || v == 4 || v == 6)
                        hipExtLaunchKernelGGL(k_spin, dim3(64), dim3(256), 0, s, nullptr, e, 0, buf, spin);
                    else
                        hipLaunchKernelGGL(k_spin, dim3(64), dim3(256), 0, s, buf, spin);
                    if (v == 1 || v == 3) CK(hipEventRecord(e, s));
                    if (v == 3 || v == 4 || v == 6) CK(hipStreamWaitEvent(side, e, 0));
                    if (v == 6) {
                        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, side, buf + 65536, 10);
                        CK(hipEventRecord(e2, side));
                    }
                    hipLaunchKernelGGL(k_spin, dim3(64), dim3(256), 0, s, buf, spin);
                    if (v == 5 || v == 6) CK(hipStreamWaitEvent(s, e2, 0));
                }
                CK(hipStreamSynchronize(s));
                CK(hipStreamSynchronize(side));
                auto t1 = std::chrono::steady_clock::now();
                reps.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count() / iters);
            }
            std::sort(reps.begin(), reps.end());
            printf("%-8s %-14s %8.2f us/iter\n", fname[fi], names[v], reps[2]);
        }
    }
    return 0;
}
