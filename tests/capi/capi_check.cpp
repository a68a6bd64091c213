// A C++ consumer of the C ABI (include/trlx_t5_amd.h) with no Python and no torch: the
// boundary a maintainer binds from another host language, exercised end to end.
//
// One PPO step of the serial schedule through the fused entry points on the current HIP
// device — trlx_ppo_experience_fused (policy + reference rows, KL reward, GAE, whitening
// moments) and trlx_ppo_loss_fused (new-policy rows, PPO loss + 13 stats, dlogits, dvalues) —
// against a double-precision host restatement of the reference arithmetic written here:
//   logprobs_from_logits            trlx/utils/modeling.py:37-41
//   KL-penalised reward             trlx/orchestrator/ppo_orchestrator.py:163-167
//   get_advantages_and_returns      trlx/model/nn/ppo_models.py:121-139 (whiten: modeling.py:24-34,
//                                   torch.var_mean's unbiased variance outside torch.distributed)
//   PPOConfig.loss + its autograd   ppo_models.py:141-199
// Test infrastructure (tests/test_gpu_capi.py runs it); built by `make -C tests/capi`.
// Exit status 0 and "capi_check ok" on success.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "trlx_t5_amd.h"

#define HIP_OK(x)                                                                        \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));          \
            std::exit(2);                                                                \
        }                                                                                \
    } while (0)
#define TRLX_OK_(x)                                                                      \
    do {                                                                                 \
        int s_ = (x);                                                                    \
        if (s_ != TRLX_OK) {                                                             \
            std::fprintf(stderr, "%s failed (%d): %s\n", #x, s_, trlx_last_error());     \
            std::exit(3);                                                                \
        }                                                                                \
    } while (0)

static uint16_t to_bf16(float f) {  // round to nearest even
    uint32_t u;
    std::memcpy(&u, &f, 4);
    u += 0x7fffu + ((u >> 16) & 1u);
    return uint16_t(u >> 16);
}
static double from_bf16(uint16_t h) {
    const uint32_t u = uint32_t(h) << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

template <class T>
static T* dev_copy(const std::vector<T>& h) {
    T* d = nullptr;
    HIP_OK(hipMalloc(&d, h.size() * sizeof(T)));
    HIP_OK(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    return d;
}
template <class T>
static std::vector<T> host_copy(const T* d, size_t n) {
    std::vector<T> h(n);
    HIP_OK(hipMemcpy(h.data(), d, n * sizeof(T), hipMemcpyDeviceToHost));
    return h;
}
template <class T>
static T* dev_alloc(size_t n) {
    T* d = nullptr;
    HIP_OK(hipMalloc(&d, n * sizeof(T)));
    HIP_OK(hipMemset(d, 0, n * sizeof(T)));
    return d;
}

static int g_fail = 0;
static void check(const char* what, double got, double want, double rtol, double atol) {
    if (!(std::fabs(got - want) <= atol + rtol * std::fabs(want))) {
        if (g_fail < 20) std::fprintf(stderr, "MISMATCH %s: got %.9g want %.9g\n", what, got, want);
        ++g_fail;
    }
}

// log_softmax(row)[y] and the softmax row (double)
static double row_logprob(const uint16_t* x, int64_t V, int64_t y, std::vector<double>* p) {
    double m = -INFINITY;
    for (int64_t j = 0; j < V; ++j) m = std::fmax(m, from_bf16(x[j]));
    double s = 0.0;
    for (int64_t j = 0; j < V; ++j) s += std::exp(from_bf16(x[j]) - m);
    const double lse = m + std::log(s);
    if (p) {
        p->resize(V);
        for (int64_t j = 0; j < V; ++j) (*p)[j] = std::exp(from_bf16(x[j]) - lse);
    }
    return from_bf16(x[y]) - lse;
}

int main() {
    const int64_t B = 6, T = 13, V = 1031;
    const float beta = 0.05f, gamma = 1.0f, lam = 0.95f, clip = 0.2f, clipv = 0.2f, vf_coef = 1.0f;
    const int64_t N = B * T;
    std::mt19937_64 rng(1234);
    std::normal_distribution<float> nrm(0.0f, 1.0f);
    std::uniform_real_distribution<float> uni(-12.0f, 12.0f);
    std::vector<uint16_t> logits(N * V), ref_logits(N * V), new_logits(N * V);
    for (int64_t i = 0; i < N * V; ++i) {
        const float x = 2.0f * nrm(rng);
        logits[i] = to_bf16(x);
        ref_logits[i] = to_bf16(x + 0.1f * nrm(rng));
        new_logits[i] = to_bf16(x + 0.05f * nrm(rng));
    }
    std::vector<int64_t> labels(N);
    for (int64_t i = 0; i < N; ++i) labels[i] = int64_t(rng() % uint64_t(V));
    labels[0] = 0;
    labels[N - 1] = V - 1;
    std::vector<float> old_values(N), values(N), scores(B);
    for (int64_t i = 0; i < N; ++i) {
        old_values[i] = nrm(rng);
        values[i] = old_values[i] + 0.3f * nrm(rng);
    }
    for (int64_t b = 0; b < B; ++b) scores[b] = uni(rng);

    // ---- device step through the C ABI (stream 0 = the default stream)
    uint16_t *d_x = dev_copy(logits), *d_rx = dev_copy(ref_logits), *d_nx = dev_copy(new_logits);
    int64_t* d_y = dev_copy(labels);
    float *d_ov = dev_copy(old_values), *d_v = dev_copy(values), *d_sc = dev_copy(scores);
    float *d_lp = dev_alloc<float>(N), *d_rlp = dev_alloc<float>(N), *d_rew = dev_alloc<float>(N);
    float *d_adv = dev_alloc<float>(N), *d_ret = dev_alloc<float>(N), *d_lpn = dev_alloc<float>(N);
    float *d_dv = dev_alloc<float>(N), *d_loss = dev_alloc<float>(1), *d_stats = dev_alloc<float>(TRLX_PPO_STATS);
    double* d_mom = dev_alloc<double>(TRLX_MOMENT_SLOTS);
    uint16_t* d_dx = dev_alloc<uint16_t>(N * V);
    uint8_t* d_ws = dev_alloc<uint8_t>(size_t(trlx_ppo_workspace_bytes(B, T)));  // zero-filled once
    TRLX_OK_(trlx_ppo_experience_fused(d_x, d_rx, TRLX_BF16, B, T, V, T * V, V, d_y, T, 1, d_ov, TRLX_F32, d_sc,
                                       nullptr, nullptr, beta, gamma, lam, d_lp, d_rlp, d_rew, d_adv, d_ret, TRLX_F32,
                                       d_mom, d_ws, nullptr));
    TRLX_OK_(trlx_ppo_loss_fused(d_nx, TRLX_BF16, B, T, V, T * V, V, d_y, T, 1, d_lp, TRLX_F32, d_adv, d_mom,
                                 /*unbiased=*/1, nullptr, d_v, TRLX_F32, d_ov, TRLX_F32, d_ret, TRLX_F32, clip, clipv,
                                 vf_coef, d_lpn, d_dx, T * V, V, d_dv, d_loss, d_stats, d_ws, nullptr));
    HIP_OK(hipDeviceSynchronize());
    const std::vector<float> lp = host_copy(d_lp, N), rew = host_copy(d_rew, N), ret = host_copy(d_ret, N);
    const std::vector<float> lpn = host_copy(d_lpn, N), dv = host_copy(d_dv, N), loss = host_copy(d_loss, 1);
    const std::vector<float> stats = host_copy(d_stats, TRLX_PPO_STATS);
    const std::vector<uint16_t> dx = host_copy(d_dx, size_t(N * V));

    // ---- host restatement (double)
    std::vector<double> hlp(N), hrlp(N), hrew(N), hA(N), hret(N);
    for (int64_t i = 0; i < N; ++i) {
        hlp[i] = row_logprob(&logits[i * V], V, labels[i], nullptr);
        hrlp[i] = row_logprob(&ref_logits[i * V], V, labels[i], nullptr);
        hrew[i] = -double(beta) * (hlp[i] - hrlp[i]);
    }
    for (int64_t b = 0; b < B; ++b) {
        hrew[b * T + T - 1] += scores[b];
        double A = 0.0;
        for (int64_t t = T - 1; t >= 0; --t) {
            const double nv = t + 1 < T ? old_values[b * T + t + 1] : 0.0;
            const double delta = hrew[b * T + t] + gamma * nv - old_values[b * T + t];
            A = delta + double(gamma) * double(lam) * A;
            hA[b * T + t] = A;
            hret[b * T + t] = A + old_values[b * T + t];
        }
    }
    double mean = 0.0;
    for (int64_t i = 0; i < N; ++i) mean += hA[i];
    mean /= double(N);
    double var = 0.0;
    for (int64_t i = 0; i < N; ++i) var += (hA[i] - mean) * (hA[i] - mean);
    var /= double(N - 1);  // torch.var_mean (unbiased)
    const double rstd = 1.0 / std::sqrt(var + 1e-8);
    double pg_sum = 0.0, vf_sum = 0.0, kl_sum = 0.0;
    std::vector<double> hlpn(N), hdv(N);
    std::vector<double> p;
    for (int64_t i = 0; i < N; ++i) {
        hlpn[i] = row_logprob(&new_logits[i * V], V, labels[i], &p);
        const double Aw = (hA[i] - mean) * rstd;
        const double lr = hlpn[i] - hlp[i];
        const double ratio = std::exp(lr);
        const double cr = std::fmin(std::fmax(ratio, 1.0 - clip), 1.0 + clip);
        const double pg1 = -Aw * ratio, pg2 = -Aw * cr;
        pg_sum += std::fmax(pg1, pg2);
        kl_sum += (ratio - 1.0) - lr;
        // d pg_loss / d lp_new (torch.maximum: 1/2-1/2 on ties; clamp passes at its bounds)
        const double g1 = pg1 == pg2 ? 0.5 : (pg1 > pg2 ? 1.0 : 0.0), g2 = pg1 == pg2 ? 0.5 : 1.0 - g1;
        const double inr = (ratio >= 1.0 - clip && ratio <= 1.0 + clip) ? 1.0 : 0.0;
        const double dlp = (g1 * -Aw + g2 * -Aw * inr) * ratio / double(N);
        for (int64_t j = 0; j < V; ++j) {
            const double want = dlp * ((j == labels[i] ? 1.0 : 0.0) - p[j]);
            if (j == labels[i] || std::fabs(want) > 1e-7)  // relative check where it is representable
                check("dlogits", from_bf16(dx[i * V + j]), want, 1.6e-2, 1e-8);
        }
        const double v = values[i], ov = old_values[i], R = hret[i];
        const double vc = std::fmin(std::fmax(v, ov - clipv), ov + clipv);
        const double e1 = (v - R) * (v - R), e2 = (vc - R) * (vc - R);
        vf_sum += std::fmax(e1, e2);
        const double h1 = e1 == e2 ? 0.5 : (e1 > e2 ? 1.0 : 0.0), h2 = e1 == e2 ? 0.5 : 1.0 - h1;
        const double vin = (v >= ov - clipv && v <= ov + clipv) ? 1.0 : 0.0;
        hdv[i] = double(vf_coef) * 0.5 / double(N) * (h1 * 2.0 * (v - R) + h2 * 2.0 * (vc - R) * vin);
    }
    const double hloss = pg_sum / double(N) + double(vf_coef) * 0.5 * vf_sum / double(N);

    for (int64_t i = 0; i < N; ++i) {
        check("lp", lp[i], hlp[i], 1e-5, 1e-5);
        check("rewards", rew[i], hrew[i], 1e-5, 1e-5);
        check("returns", ret[i], hret[i], 1e-5, 2e-5);
        check("lp_new", lpn[i], hlpn[i], 1e-5, 1e-5);
        check("dvalues", dv[i], hdv[i], 1e-5, 1e-8);
    }
    check("loss", loss[0], hloss, 1e-4, 1e-6);
    check("stats[0] total_loss", stats[0], hloss, 1e-4, 1e-6);
    check("stats[8] approx_kl", stats[8], kl_sum / double(N), 1e-3, 1e-7);
    for (void* q : {(void*)d_x, (void*)d_rx, (void*)d_nx, (void*)d_y, (void*)d_ov, (void*)d_v, (void*)d_sc,
                    (void*)d_lp, (void*)d_rlp, (void*)d_rew, (void*)d_adv, (void*)d_ret, (void*)d_lpn, (void*)d_dv,
                    (void*)d_loss, (void*)d_stats, (void*)d_mom, (void*)d_dx, (void*)d_ws})
        HIP_OK(hipFree(q));
    if (g_fail) {
        std::fprintf(stderr, "capi_check: %d mismatches\n", g_fail);
        return 1;
    }
    std::printf("capi_check ok: B=%lld T=%lld V=%lld loss %.6f (host %.6f)\n", (long long)B, (long long)T,
                (long long)V, loss[0], hloss);
    return 0;
}
