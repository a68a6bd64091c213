// Standalone entry points of the device-resident controller state:
// state init, score moments for the cross-rank all-reduce, the score-side control
// (RunningMoments.update + scale + clip, ppo_orchestrator.py:96-112) and the KL controller
// update (ppo_models.py:26-58).  All are single-workgroup launches over small vectors; the
// fused PPO step folds the same device code into its rollout tails (row_tails.h) instead.
#include <hip/hip_ext.h>

#include "ctl_state.h"

namespace trlx {

constexpr int kCtlThreads = 1024;

__global__ void k_ctl_init(double* st, double beta, double ref_mean, double ref_std, int ref_set) {
    const int k = threadIdx.x;
    if (k >= TRLX_CTL_SLOTS) return;
    double v = 0.0;
    switch (k) {
        case TRLX_CTL_MEAN: v = 0.0; break;
        case TRLX_CTL_VAR: v = 1.0; break;
        case TRLX_CTL_STD: v = 1.0; break;
        case TRLX_CTL_COUNT: v = 1e-24; break;
        case TRLX_CTL_REF_MEAN: v = ref_mean; break;
        case TRLX_CTL_REF_STD: v = ref_std; break;
        case TRLX_CTL_REF_SET: v = ref_set ? 1.0 : 0.0; break;
        case TRLX_CTL_KL_COEF: v = beta; break;
        default: v = 0.0;
    }
    st[k] = v;
}

__global__ __launch_bounds__(kCtlThreads) void k_score_moments(const float* x, int n, double* out) {
    __shared__ double red[3 * (kCtlThreads / kWave)];
    double s = 0.0, ss = 0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const double v = double(x[i]);
        s += v;
        ss = fma(v, v, ss);
    }
    const double m[3] = {s, ss, 0.0};
    const double r = block_sum_multi<3>(m, red);
    if (threadIdx.x < 2) out[threadIdx.x] = r;
    if (threadIdx.x == 2) out[2] = double(n);
    if (threadIdx.x == 3) out[3] = 0.0;
}

__global__ __launch_bounds__(kCtlThreads) void k_score_ctl(const float* x, int n, ScoreCtlArgs c, float* out) {
    float div, beta;
    score_ctl_block(c, x, n, true, div, beta);
    for (int i = threadIdx.x; i < n; i += blockDim.x) out[i] = score_transform(x[i], div, c.clip);
}

__global__ void k_moments_merge(const double* state_in, double* state_out, const double* moments) {
    if (threadIdx.x != 0) return;
    RunStats r;
    r.load(state_in);
    running_merge_global(r, moments);
    for (int k = 0; k < TRLX_CTL_SLOTS; ++k) state_out[k] = state_in[k];
    r.store(state_out);
}

__global__ void k_kl_ctl(KlCtlArgs k, const float* approx_kl) {
    if (threadIdx.x == 0) kl_ctl_apply(k, *approx_kl);
}

}  // namespace trlx

using namespace trlx;

extern "C" int trlx_ctl_init(double* state, double init_kl_coef, double ref_mean, double ref_std, int ref_set,
                             void* stream) {
    TRLX_REQUIRE(state, TRLX_ERR_ARG, "NULL controller state");
    hipLaunchKernelGGL(k_ctl_init, dim3(1), dim3(kWave), 0, (hipStream_t)stream, state, init_kl_coef, ref_mean,
                       ref_std, ref_set);
    return check_launch("k_ctl_init");
}

extern "C" int trlx_score_moments(const void* scores, int dtype, int64_t n, double* moments, void* stream) {
    TRLX_REQUIRE(n > 0 && n < (1LL << 31), TRLX_ERR_SHAPE, "bad score count %lld", (long long)n);
    TRLX_REQUIRE(dtype == TRLX_F32, TRLX_ERR_DTYPE, "scores must be fp32");
    TRLX_REQUIRE(scores && moments, TRLX_ERR_ARG, "NULL argument to trlx_score_moments");
    hipLaunchKernelGGL(k_score_moments, dim3(1), dim3(kCtlThreads), 0, (hipStream_t)stream,
                       static_cast<const float*>(scores), int(n), moments);
    return check_launch("k_score_moments");
}

extern "C" int trlx_score_moments_signal(const void* scores, int dtype, int64_t n, double* moments, void* stream,
                                         void* done_event) {
    TRLX_REQUIRE(n > 0 && n < (1LL << 31), TRLX_ERR_SHAPE, "bad score count %lld", (long long)n);
    TRLX_REQUIRE(dtype == TRLX_F32, TRLX_ERR_DTYPE, "scores must be fp32");
    TRLX_REQUIRE(scores && moments && done_event, TRLX_ERR_ARG, "NULL argument to trlx_score_moments_signal");
    // the event rides the kernel's own dispatch (its completion signal): no marker packet
    // between this launch and the next one on the stream
    hipExtLaunchKernelGGL(k_score_moments, dim3(1), dim3(kCtlThreads), 0, (hipStream_t)stream, nullptr,
                          (hipEvent_t)done_event, 0, static_cast<const float*>(scores), int(n), moments);
    return check_launch("k_score_moments");
}

extern "C" int trlx_score_ctl_update(const void* scores, int dtype, int64_t n, const trlx_score_ctl* ctl,
                                     void* scores_out, int out_dtype, void* stream) {
    TRLX_REQUIRE(n > 0 && n < (1LL << 31), TRLX_ERR_SHAPE, "bad score count %lld", (long long)n);
    TRLX_REQUIRE(dtype == TRLX_F32 && out_dtype == TRLX_F32, TRLX_ERR_DTYPE, "scores must be fp32");
    TRLX_REQUIRE(scores && scores_out && ctl && ctl->state_in && ctl->state_out, TRLX_ERR_ARG,
                 "NULL argument to trlx_score_ctl_update");
    TRLX_REQUIRE(ctl->scale_mode >= TRLX_SCALE_NONE && ctl->scale_mode <= TRLX_SCALE_REF, TRLX_ERR_ARG,
                 "bad scale_mode %d", ctl->scale_mode);
    ScoreCtlArgs c = {};
    c.state_in = ctl->state_in; c.state_out = ctl->state_out; c.global_mom = ctl->global_moments;
    c.scale_mode = ctl->scale_mode; c.clip = ctl->cliprange_reward;
    hipLaunchKernelGGL(k_score_ctl, dim3(1), dim3(kCtlThreads), 0, (hipStream_t)stream,
                       static_cast<const float*>(scores), int(n), c, static_cast<float*>(scores_out));
    return check_launch("k_score_ctl");
}

extern "C" int trlx_score_moments_merge(const double* state_in, double* state_out, const double* moments,
                                        void* stream) {
    TRLX_REQUIRE(state_in && state_out && moments, TRLX_ERR_ARG, "NULL argument to trlx_score_moments_merge");
    hipLaunchKernelGGL(k_moments_merge, dim3(1), dim3(kWave), 0, (hipStream_t)stream, state_in, state_out, moments);
    return check_launch("k_moments_merge");
}

extern "C" int trlx_kl_ctl_update(const trlx_kl_ctl* kl, const float* approx_kl, void* stream) {
    TRLX_REQUIRE(kl && kl->state && approx_kl, TRLX_ERR_ARG, "NULL argument to trlx_kl_ctl_update");
    TRLX_REQUIRE(!kl->adaptive || (kl->target != 0.0 && kl->horizon != 0.0), TRLX_ERR_ARG,
                 "adaptive KL control needs target and horizon");
    KlCtlArgs k = {};
    k.state = kl->state; k.adaptive = kl->adaptive; k.target = kl->target; k.horizon = kl->horizon;
    k.n_steps = double(kl->n_steps);
    hipLaunchKernelGGL(k_kl_ctl, dim3(1), dim3(kWave), 0, (hipStream_t)stream, k, approx_kl);
    return check_launch("k_kl_ctl");
}
