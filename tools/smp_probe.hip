// Phase timing of k_ilql_sample (wall_clock64 stamps, 100 MHz) on synthetic rows.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -DTRLX_SMP_PROF
//        -Iinclude -Itrlx-t5_amd/csrc tools/smp_probe.hip trlx-t5_amd/csrc/capi.cpp -o tools/smp_probe
#include "../trlx-t5_amd/csrc/ilql_sample.hip"
#include <cstdio>
#include <cstring>
#include <vector>

int main(int argc, char** argv) {
    const int64_t B = argc > 1 ? atoll(argv[1]) : 32, V = argc > 2 ? atoll(argv[2]) : 50257;
    const int bf16 = argc > 3 ? atoi(argv[3]) : 0;
    const int topk = argc > 4 ? atoi(argv[4]) : 20;
    const size_t es = bf16 ? 2 : 4;
    std::vector<float> hf(B * V);
    uint32_t st = 12345;
    for (auto& x : hf) { st = st * 1664525u + 1013904223u; x = float(st >> 8) / 16777216.f * 8.f - 4.f; }
    std::vector<uint16_t> hb(B * V);
    for (size_t i = 0; i < hb.size(); ++i) { uint32_t u; std::memcpy(&u, &hf[i], 4); hb[i] = uint16_t(u >> 16); }
    void *lg, *q0, *q1; float *vs, *u; int64_t* out;
    hipMalloc(&lg, B * V * es); hipMalloc(&q0, B * V * es); hipMalloc(&q1, B * V * es);
    hipMalloc(&vs, B * 4); hipMalloc(&u, B * 4); hipMalloc(&out, B * 8);
    const void* src = bf16 ? (const void*)hb.data() : (const void*)hf.data();
    hipMemcpy(lg, src, B * V * es, hipMemcpyHostToDevice);
    hipMemcpy(q0, src, B * V * es, hipMemcpyHostToDevice);
    hipMemcpy(q1, src, B * V * es, hipMemcpyHostToDevice);
    hipMemset(vs, 0, B * 4); hipMemset(u, 0, B * 4);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int rep = 0; rep < 5; ++rep) {
        hipEventRecord(e0, 0);
        int rc = trlx_ilql_sample(lg, V, q0, V, q1, V, bf16 ? TRLX_BF16 : TRLX_F32, vs, nullptr, 0, nullptr, B, V,
                                  1.f, topk, 1.f, u, out, nullptr, 50256, 0);
        hipEventRecord(e1, 0);
        hipDeviceSynchronize();
        float ms; hipEventElapsedTime(&ms, e0, e1);
        static uint64_t h[4096][12];
        hipMemcpyFromSymbol(h, HIP_SYMBOL(g_smp_prof), sizeof(uint64_t) * 12 * B);
        double acc[8] = {}, ncand = 0;
        auto d = [&](int b, int i, int j) { return double(h[b][j] - h[b][i]) * 10e-3; };
        for (int b = 0; b < B; ++b) {
            acc[0] += d(b, 0, 1); acc[1] += d(b, 1, 2); acc[2] += d(b, 2, 3);
            acc[3] += d(b, 3, 7); acc[4] += d(b, 7, 8); acc[5] += d(b, 8, 4); acc[6] += d(b, 4, 6);
            ncand += double(h[b][9]);
        }
        printf("rc=%d event %.1f us | phases (us, mean over rows): load %.1f lse %.1f score %.1f t0 %.1f "
               "append %.1f select %.1f draw %.1f | candidates %.0f\n", rc, ms * 1e3, acc[0] / B, acc[1] / B,
               acc[2] / B, acc[3] / B, acc[4] / B, acc[5] / B, acc[6] / B, ncand / B);
        memset(h, 0, sizeof(h));
        hipMemcpyToSymbol(HIP_SYMBOL(g_smp_prof), h, sizeof(uint64_t) * 12 * B);
    }
    return 0;
}
