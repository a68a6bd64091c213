// Device-resident controller state of the PPO loop: the reward
// RunningMoments (trlx/utils/modeling.py:72-104), the score scale / clip of the
// orchestrator (trlx/orchestrator/ppo_orchestrator.py:96-112) and the KL coefficient of
// AdaptiveKLController / FixedKLController (trlx/model/nn/ppo_models.py:26-58) live in one
// fp64 record in HBM (TRLX_CTL_SLOTS doubles, layout in trlx_t5_amd.h), so a PPO step reads
// and advances them in-stream with no host synchronisation.
//
// The reference keeps these as Python scalars / 0-d tensors and reads them back every
// chunk (`.item()`-style host round trips in the KL controller, RunningMoments attributes
// as Python numbers).  Here the scalar arithmetic runs in fp64 on thread 0 of whichever
// block needs it; the batch moments are block reductions over the (small) score vector.
#pragma once
#include "common.h"

namespace trlx {

struct ScoreCtlArgs {
    const double* state_in;    // [TRLX_CTL_SLOTS]
    double* state_out;         // [TRLX_CTL_SLOTS] (written by one block only)
    const double* global_mom;  // {Σx, Σx², n} over all ranks, or NULL (local = global)
    int scale_mode;            // TRLX_SCALE_*
    float clip;                // cliprange_reward (0: no clip)
    int lag;                   // 1: global_mom holds the PREVIOUS batch's moments (merged now; NULL: nothing
                               // to merge yet) -- the pipelined schedule without running-std scaling
};

// The RunningMoments slots of the record, as scalars (a thread holds six doubles instead of
// the whole record: the merge also runs inside the loss rows kernel, at 64 VGPRs).
struct RunStats {
    double mean, var, std, count, bmean, bstd;
    __device__ __forceinline__ void load(const double* st) {
        mean = st[TRLX_CTL_MEAN]; var = st[TRLX_CTL_VAR]; std = st[TRLX_CTL_STD]; count = st[TRLX_CTL_COUNT];
        bmean = st[TRLX_CTL_BATCH_MEAN]; bstd = st[TRLX_CTL_BATCH_STD];
    }
    __device__ __forceinline__ void store(double* st) const {
        st[TRLX_CTL_MEAN] = mean; st[TRLX_CTL_VAR] = var; st[TRLX_CTL_STD] = std; st[TRLX_CTL_COUNT] = count;
        st[TRLX_CTL_BATCH_MEAN] = bmean; st[TRLX_CTL_BATCH_STD] = bstd;
    }
};

// RunningMoments.update's merge (modeling.py:91-102, term for term) of batch moments
// (n, mean, biased var) into the record; also the batch statistics it returns.
__device__ __forceinline__ void running_merge(RunStats& r, double xn, double xm, double xv) {
    const double delta = xm - r.mean;
    const double cnt = r.count;
    const double tot = cnt + xn;
    const double new_sum = xv * xn;
    const double old_sum = r.var * cnt + delta * delta * cnt * xn / tot;
    r.mean += delta * xn / tot;
    r.var = (old_sum + new_sum) / tot;
    r.std = sqrt(r.var * tot / (tot - 1.0));
    r.count = tot;
    r.bmean = xm;
    r.bstd = sqrt(xv * xn / (xn - 1.0));
}
// the same from an all-reduced {Σx, Σx², n} record (get_global_statistics, biased variance)
__device__ __forceinline__ void running_merge_global(RunStats& r, const double* gm) {
    const double xn = gm[2];
    const double xm = gm[0] / xn;
    running_merge(r, xn, xm, fmax(gm[1] - gm[0] * xm, 0.0) / xn);
}

struct KlCtlArgs {
    double* state;  // NULL: no KL update
    int adaptive;
    double target, horizon, n_steps;
};

// Divide-and-clip of one score (ppo_orchestrator.py:104-112): fp32 division by the fp32
// scale (the reference divides fp32 tensors), then torch.clip.  div == 0 => no scaling.
__device__ __forceinline__ float score_transform(float x, float div, float clip) {
    if (div != 0.0f) x = __fdiv_rn(x, div);
    if (clip != 0.0f) x = fminf(fmaxf(x, -clip), clip);
    return x;
}

// RunningMoments.update + the reference-statistics bookkeeping + the scale choice, for
// the whole block (every thread must call it; it contains barriers).  Batch moments of
// scores[0, n): two fp64 passes (mean, then Σ(x - mean)²) -> the local statistics; the
// running merge uses global_mom when given (get_global_statistics across ranks,
// modeling.py:9-21, biased variance) and the local ones otherwise (torch.var_mean,
// unbiased=False, modeling.py:86-87).  First call with ref unset: ref_mean / ref_std =
// scores.mean(), scores.std() of the LOCAL batch (ppo_orchestrator.py:96-98, unbiased).
// Outputs (all threads): the fp32 divisor for score_transform (0 = none) and beta.
// When `writer`, thread 0 stores the advanced record to state_out.
// nthr (0 = blockDim.x): the threads that take scores (the GAE block is 256 threads wide in
// its arithmetic even inside a 512-thread loss rows workgroup: same partial sums, same bits).
__device__ __forceinline__ void score_ctl_block(const ScoreCtlArgs& c, const float* scores, int n, bool writer,
                                                float& div, float& beta, int nthr = 0) {
    __shared__ double s_red[2 * (1024 / kWave)];
    __shared__ float s_out[2];
    const int nw = blockDim.x / kWave;
    const int stride = nthr ? nthr : int(blockDim.x);
    const int i0 = int(threadIdx.x) < stride ? int(threadIdx.x) : n;
    double s = 0.0;
    #pragma unroll 1
    for (int i = i0; i < n; i += stride) s += double(scores[i]);
    s = block_sum_d(s, s_red);
    const double lmean = s / double(n);
    double m2 = 0.0;
    #pragma unroll 1
    for (int i = i0; i < n; i += stride) {
        const double d = double(scores[i]) - lmean;
        m2 = fma(d, d, m2);
    }
    m2 = block_sum_d(m2, s_red + nw);
    if (threadIdx.x == 0) {
        const double* si = c.state_in;
        RunStats r;
        r.load(si);
        if (c.global_mom)
            running_merge_global(r, c.global_mom);  // lag: the previous batch's, all-reduced
        else if (!c.lag)
            running_merge(r, double(n), lmean, m2 / double(n));
        double ref_mean = si[TRLX_CTL_REF_MEAN], ref_std = si[TRLX_CTL_REF_STD];
        const bool set_ref = si[TRLX_CTL_REF_SET] == 0.0;
        if (set_ref) {
            ref_mean = lmean;
            ref_std = sqrt(m2 / (double(n) - 1.0));
        }
        float d = 0.0f;
        if (c.scale_mode == TRLX_SCALE_RUNNING) d = float(r.std);
        else if (c.scale_mode == TRLX_SCALE_REF) d = float(ref_std);
        s_out[0] = d;
        s_out[1] = float(si[TRLX_CTL_KL_COEF]);
        if (writer) {  // (state_out may alias state_in: every slot read above is read before)
            double* so = c.state_out;
#pragma unroll 1
            for (int k = 0; k < TRLX_CTL_SLOTS; ++k) so[k] = si[k];  // the slots not advanced here
            r.store(so);
            so[TRLX_CTL_REF_MEAN] = ref_mean;
            so[TRLX_CTL_REF_STD] = ref_std;
            so[TRLX_CTL_REF_SET] = 1.0;
        }
    }
    __syncthreads();
    div = s_out[0];
    beta = s_out[1];
}

// AdaptiveKLController.update (ppo_models.py:38-44) in fp64 on one thread:
//   beta *= 1 + clip(current/target - 1, -0.2, 0.2) * n_steps / horizon
// np.clip propagates NaN, so the clamp is written with comparisons (fmin/fmax would drop it).
__device__ __forceinline__ void kl_ctl_apply(const KlCtlArgs& k, float approx_kl) {
    if (!k.state) return;
    const double cur = double(approx_kl);
    if (k.adaptive) {
        double err = cur / k.target - 1.0;
        err = err < -0.2 ? -0.2 : (err > 0.2 ? 0.2 : err);
        const double mult = 1.0 + err * k.n_steps / k.horizon;
        k.state[TRLX_CTL_KL_COEF] = k.state[TRLX_CTL_KL_COEF] * mult;
    }
    k.state[TRLX_CTL_KL_UPDATES] += 1.0;
    k.state[TRLX_CTL_LAST_KL] = cur;
}

}  // namespace trlx
