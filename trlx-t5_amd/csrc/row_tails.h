// Rollout-level [T]-vector work of the fused step, one wavefront per rollout.
//
// The vocab-row kernels (one workgroup per token row) leave per-token results in HBM;
// these small kernels then run one wave per rollout (a lane per token, 64-token chunks):
//   k_rollout_gae   KL-penalised rewards + GAE (lane-parallel suffix scan) + the
//                   whitening moments {Σ A, Σ A², n, Σ mask}
//   k_rollout_loss  fp64 sums of the per-token PPO loss terms -> loss + 13 stats
// Each block publishes one fp64 record; the block that arrives last reduces them in fixed
// order (common.h publish_record_last: write-through `sc1` records + one returned atomic,
// no fences), so each is ONE launch of ~B/4 blocks.  An earlier version folded this work
// into the row kernels' tails with a per-rollout arrival ticket; every row workgroup then
// held its CU slot for a write-through store + returned atomic (~2 us), which cost 10-15%
// of the streaming kernels' bandwidth (measured) — a separate launch is cheaper.
#pragma once
#include "ctl_state.h"
#include "ppo_math.h"

namespace trlx {

constexpr int kRolloutThreads = 256;                 // 4 waves = 4 rollouts per block
constexpr int kRolloutsPerBlock = kRolloutThreads / kWave;
constexpr int kTokRec = 12;                          // floats per token record (11 used)

// Wave-wide fixed-order (butterfly) sum; every lane ends with the total.
__device__ __forceinline__ double wave_allsum_d(double v) {
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) v += __shfl_xor(v, off, kWave);
    return v;
}

// Workspace carve-up (16-B aligned sections), see trlx_ppo_workspace_bytes:
//   tickets : uint32[4]                    (zero before first use; re-armed in-kernel)
//   gae_rec : double[nblk][8]              per-block moments (4 used unless split-beta)
//   loss_rec: double[nblk][16]             per-block loss sums
//   tokrec  : float[B*T][kTokRec]          per-token loss terms
struct Workspace {
    unsigned* tickets;
    double* gae_rec;
    double* loss_rec;
    float* tokrec;
    int* order;       // a ragged batch's experience-row dispatch order (vocab_rows.hip k_ragged_order)
};

// ------------------------------------------------------------------ GAE per rollout
struct GaeRolloutArgs {
    int B, T;
    const float* lp;          // [B,T] policy logprobs (fp32)
    const float* ref_lp;      // [B,T] reference logprobs (fp32)
    const void* values;       // [B,T] old values
    int v_dtype;
    const float* scores;      // [B] or NULL
    const int64_t* lengths;   // [B] or NULL
    const int64_t* mask;      // [B,T] loss mask or NULL
    float neg_beta, gamma, gl;
    float* rewards;           // [B,T] fp32 out
    float* adv;               // [B,T] fp32 out (unwhitened)
    void* ret;                // [B,T] out
    int ret_dtype;
    double* stats;            // [4] out ([8] split-beta)
    Workspace ws;
    int has_ctl;              // score/beta control from the device state (ctl_state.h)
    ScoreCtlArgs ctl;
    // split-beta GAE (k_rollout_gae<true>): beta-free outputs, beta applied by the loss rows
    float* adv_kl;            // [B,T] out: GAE suffix sums of the KL term (the "A_k" part)
    float* rew_kl;            // [B,T] out: lp - ref_lp (0 past the rollout's length)
    float* rew_score;         // [B,T] out: score term (the score at the last column, -0.0 before it, 0 past it)
    // optional: whitening coefficients of the PREVIOUS batch, folded into this launch
    const double* prev_stats; // [8] split record of that batch (all-reduced) or NULL
    float* prev_coef;         // [4] out {mu, rstd, beta, 0}
    int prev_unbiased;
    float host_beta;          // beta without device controller state
};

// Split-beta whitening coefficients: the KL-penalised reward is r = score_t - beta*kl_t and
// GAE is linear in r, so A = A0 - beta*Ak with A0 the GAE of the score + value terms and Ak
// the discounted KL sums.  The split record {Σ A0, Σ A0², n, Σ Ak, Σ A0·Ak, Σ Ak², Σ mask, 0}
// gives Σ A = Σ A0 - beta Σ Ak and Σ A² = Σ A0² - 2 beta Σ A0·Ak + beta² Σ Ak² in fp64, then
// the same {sum, sumsq, n} whitening as the unsplit path (modeling.py:24-34).
__device__ __forceinline__ void whiten_split_coeffs(const double* st, int unbiased, float beta, float& mu, float& rstd) {
    const double b = double(beta);
    const double rec[3] = {fma(-b, st[3], st[0]), fma(b * b, st[5], fma(-2.0 * b, st[4], st[1])), st[2]};
    whiten_coeffs(rec, unbiased, mu, rstd);
}
__device__ __forceinline__ void whiten_coef_split(const double* st, int unbiased, float beta, float* coef) {
    float mu, rstd;
    whiten_split_coeffs(st, unbiased, beta, mu, rstd);
    coef[0] = mu;
    coef[1] = rstd;
    coef[2] = beta;
    coef[3] = 0.0f;
}

// KL reward (ppo_orchestrator.py:164-167, score on the last valid column) and GAE
// (ppo_models.py:128-136) for one rollout: the suffix recurrence A_t = δ_t + c·A_{t+1} as a
// lane-parallel scan (log2 64 steps) per 64-token chunk from the end, the carry
// A_{chunk end} entering with weight c^(n).  fp32 re-association vs the reference's
// sequential loop: ~1e-7 relative.
//
// SPLIT (split-beta, the pipelined DP schedule): beta is not needed here.  The scan runs
// twice on the same lanes — A0 over δ0 = score_t + γ·V_{t+1} − V_t and Ak over kl_t — and
// the block record carries the split moments (whiten_coef_split); rewards, returns and
// whitening are finished by the loss rows once beta is known, so this launch no longer
// waits for the previous batch's KL-controller update.  Block 0 may also emit the
// previous batch's whitening coefficients (prev_stats -> prev_coef) with the beta the
// state holds now.
// One block of the GAE launch: rollouts [blk*4, blk*4 + 4) of nblk blocks.  The block is
// kRolloutThreads (4 waves) wide in its arithmetic whatever blockDim.x is (>= 256, a multiple
// of 64): the split GAE also runs as the first workgroups of a loss rows launch
// (k_vocab_rows<kPpo>, trlx_ppo_loss_rows_split_gae), whose 512-thread workgroups leave waves
// 4.. idle; their zero partials join the fixed-order sums without changing them, so both
// forms give the same bits.  `red` holds (blockDim.x / 64) * 8 doubles.
template <bool SPLIT>
__device__ __forceinline__ void gae_block(const GaeRolloutArgs& e, int blk, int nblk, double* red) {
    constexpr int NS = SPLIT ? 8 : TRLX_MOMENT_SLOTS;
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = int(threadIdx.x / kWave);
    const int b = wv < kRolloutsPerBlock ? blk * kRolloutsPerBlock + wv : e.B;  // waves 4..: idle
    const int T = e.T;
    double s1 = 0.0, s2 = 0.0, sm = 0.0, cnt = 0.0, sk = 0.0, sak = 0.0, skk = 0.0;
    float neg_beta = e.neg_beta, sdiv = 0.0f, sclip = 0.0f;
    // Device controller state: with a score scale every block needs the merged statistics
    // up front (each derives the same values; block 0 stores them).  Without one (the
    // reference default, scale_reward False) the blocks only read beta and clip, and block 0
    // advances RunningMoments after its own rollouts, off the other blocks' path.
    const bool ctl_first = e.has_ctl && e.ctl.scale_mode != TRLX_SCALE_NONE;
    if (ctl_first) {
        float beta;
        score_ctl_block(e.ctl, e.scores, e.B, blk == 0, sdiv, beta, kRolloutThreads);
        neg_beta = -beta;
    } else if (e.has_ctl) {
        neg_beta = -float(e.ctl.state_in[TRLX_CTL_KL_COEF]);
    }
    if (e.has_ctl) sclip = e.ctl.clip;
    if (SPLIT && e.prev_stats && blk == 0 && threadIdx.x == 0)
        whiten_coef_split(e.prev_stats, e.prev_unbiased, e.has_ctl ? float(e.ctl.state_in[TRLX_CTL_KL_COEF]) : e.host_beta,
                          e.prev_coef);
    if (b < e.B) {
        const int len = e.lengths ? int(e.lengths[b]) : T;
        const float log2c = e.gl > 0.0f ? __log2f(e.gl) : -INFINITY;
        float carry = 0.0f, vcarry = 0.0f, kcarry = 0.0f;  // A (A0, Ak) and V just past the current chunk
        #pragma unroll 1
        for (int c0 = ((T - 1) / kWave) * kWave; c0 >= 0; c0 -= kWave) {
            const int t = c0 + lane;
            const bool ok = t < T;
            const int64_t gi = int64_t(b) * T + t;
            float v = 0.0f, r = 0.0f, kl = 0.0f, sc = 0.0f;
            if (ok && t < len) {
                v = ld_any(e.values, e.v_dtype, gi);
                kl = e.lp[gi] - e.ref_lp[gi];
                sc = -0.0f;  // x + (-0.0) == x: the loss rows' add leaves a score-free reward as is
                if (t == len - 1 && e.scores) sc = score_transform(e.scores[b], sdiv, sclip);
                if (!SPLIT) {
                    r = mul_rn(neg_beta, kl);
                    if (t == len - 1 && e.scores) r = add_rn(r, sc);
                }
            }
            float vn = __shfl_down(v, 1, kWave);
            if (lane == kWave - 1) vn = vcarry;
            const float delta = ok ? add_rn(SPLIT ? sc : r, mul_rn(e.gamma, vn)) - v : 0.0f;
            float x = delta, xk = kl, cd = e.gl;
#pragma unroll
            for (int d = 1; d < kWave; d <<= 1) {
                const float y = __shfl_down(x, d, kWave);
                if (lane + d < kWave) x = fmaf(cd, y, x);
                if (SPLIT) {
                    const float yk = __shfl_down(xk, d, kWave);
                    if (lane + d < kWave) xk = fmaf(cd, yk, xk);
                }
                cd = cd * cd;
            }
            const int end = min(c0 + kWave, T);
            const float cw = exp2_fast(float(end - t) * log2c);
            const float A = ok ? fmaf(cw, carry, x) : 0.0f;
            carry = __shfl(A, 0, kWave);
            vcarry = __shfl(v, 0, kWave);
            float Ak = 0.0f;
            if (SPLIT) {
                Ak = ok ? fmaf(cw, kcarry, xk) : 0.0f;
                kcarry = __shfl(Ak, 0, kWave);
            }
            if (ok) {
                e.adv[gi] = A;
                if (SPLIT) {
                    e.adv_kl[gi] = Ak;
                    e.rew_kl[gi] = kl;
                    e.rew_score[gi] = t < len ? sc : 0.0f;
                    sk += double(Ak);
                    sak += double(A) * double(Ak);
                    skk += double(Ak) * double(Ak);
                } else {
                    e.rewards[gi] = r;
                    st_any(e.ret, e.ret_dtype, gi, add_rn(A, v));
                }
                s1 += double(A);
                s2 += double(A) * double(A);
                sm += e.mask ? double(e.mask[gi]) : 1.0;
                cnt += 1.0;
            }
        }
    }
    if (e.has_ctl && !ctl_first && blk == 0) {
        float d_unused, b_unused;
        score_ctl_block(e.ctl, e.scores, e.B, true, d_unused, b_unused, kRolloutThreads);
    }
    double mine[NS];
    if constexpr (SPLIT) {  // {Σ A0, Σ A0², n, Σ Ak, Σ A0·Ak, Σ Ak², Σ mask, 0}
        mine[0] = s1; mine[1] = s2; mine[2] = cnt; mine[3] = sk; mine[4] = sak; mine[5] = skk; mine[6] = sm;
        mine[7] = 0.0;
    } else {
        mine[0] = s1; mine[1] = s2; mine[2] = cnt; mine[3] = sm;
    }
    const double rec = block_sum_multi<NS>(mine, red);
    if (publish_record_last<NS>(e.ws.gae_rec + blk * NS, rec, e.ws.tickets + 0, unsigned(nblk))) {
        __syncthreads();  // red[] reuse
        const double tot = reduce_records<NS>(e.ws.gae_rec, nblk, red, kRolloutThreads);
        if (threadIdx.x < NS) e.stats[threadIdx.x] = tot;
    }
}


template <bool SPLIT>
__global__ __launch_bounds__(kRolloutThreads) void k_rollout_gae(GaeRolloutArgs e) {
    __shared__ double red[kRolloutsPerBlock * (SPLIT ? 8 : TRLX_MOMENT_SLOTS)];
    gae_block<SPLIT>(e, int(blockIdx.x), int(gridDim.x), red);
}

// The split-beta whitening coefficients as a launch of its own (one thread): the serial
// split schedule, and the last batch of a pipelined sequence (nothing left to fold it into).
// (The two non-template kernels of this header are defined in the one translation unit that
// launches them, vocab_rows.hip; other includers define TRLX_ROW_TAILS_NO_KERNELS.)
#ifndef TRLX_ROW_TAILS_NO_KERNELS
__global__ void k_whiten_coef(const double* stats, int unbiased, const double* ctl_state, float host_beta,
                              float* coef) {
    if (threadIdx.x == 0)
        whiten_coef_split(stats, unbiased, ctl_state ? float(ctl_state[TRLX_CTL_KL_COEF]) : host_beta, coef);
}
#endif

// ------------------------------------------------------------------ loss sums per rollout
struct LossRolloutArgs {
    int B, T;
    const double* msum;       // device Σ mask (stats[3]) or NULL -> B*T
    float vf_coef;
    float* loss;              // [1] out
    float* stats;             // [13] out
    Workspace ws;
    KlCtlArgs kl;             // kl_ctl.update(approx_kl) after the stats (state NULL: none)
};

// Per-token terms of PPOConfig.loss (ppo_models.py:155-178) and d loss / d values for one
// token; thread 0 of the token's row workgroup, after its row is stored.
struct LossTokenArgs {
    const void* values;
    int v_dtype;
    const void* old_values;
    int ov_dtype;
    const void* returns;
    int r_dtype;
    float cv, vf_coef;
    float* dv;
};
// The token's value-side inputs {values, old_values, returns}; thread 0 loads them in the
// row kernel's prologue, while the row's loads are in flight, so the epilogue after the
// row store is pure arithmetic + fire-and-forget stores (a dependent load there held every
// row workgroup ~2 us longer: -7% bandwidth, measured).
__device__ __forceinline__ void loss_token_inputs(const LossTokenArgs& L, int64_t row, float* out3) {
    out3[0] = ld_any(L.values, L.v_dtype, row);
    out3[1] = ld_any(L.old_values, L.ov_dtype, row);
    out3[2] = ld_any(L.returns, L.r_dtype, row);
}
__device__ __forceinline__ void loss_token_terms(const LossTokenArgs& L, float* tokrec, int64_t row,
                                                 const PolicyTerms& pt, float m, float inv_msum, float v,
                                                 float ov, float R) {
    const float vlo = ov - L.cv, vhi = ov + L.cv;
    const float vc = fminf(fmaxf(v, vlo), vhi);
    const float e1 = v - R, e2 = vc - R;
    const float vl1 = mul_rn(e1, e1), vl2 = mul_rn(e2, e2);
    const float u = mul_rn(mul_rn(mul_rn(L.vf_coef, inv_msum), 0.5f), m);
    float h1, h2;
    if (vl1 == vl2) {  // torch.max splits ties
        h1 = u * 0.5f;
        h2 = h1;
    } else {
        h1 = vl1 > vl2 ? u : 0.0f;
        h2 = vl1 > vl2 ? 0.0f : u;
    }
    const float inr = (v >= vlo && v <= vhi) ? 1.0f : 0.0f;  // clamp passes at its bounds
    L.dv[row] = add_rn(mul_rn(mul_rn(h1, 2.0f), e1), mul_rn(mul_rn(mul_rn(h2, 2.0f), e2), inr));
    float* rec = tokrec + row * kTokRec;
    rec[0] = mul_rn(fmaxf(vl1, vl2), m);
    rec[1] = vl2 > vl1 ? 1.0f : 0.0f;
    rec[2] = (pt.ratio - 1.0f) - pt.lr;
    rec[3] = mul_rn(pt.pgmax, m);
    rec[4] = pt.pgclip ? 1.0f : 0.0f;
    rec[5] = ov;
    rec[6] = v;
    rec[7] = vl1;
    rec[8] = R;
    rec[9] = mul_rn(pt.ratio, m);
    rec[10] = m;
}

// The loss tail of one block of blockDim.x / 64 rollouts (one wave each), block `blk` of
// `nblk`: fixed-order fp64 sums of the token records, one record per block, and the block
// that arrives last emits loss + stats and applies the KL-controller update.  `red` holds
// (blockDim.x / 64) * 16 doubles.  Runs as k_rollout_loss, or as the first blocks of the
// next experience rows launch (k_vocab_rows, trlx_lsm_gather_fwd_loss_tail).
__device__ __forceinline__ void loss_tail_block(const LossRolloutArgs& L, int blk, int nblk, double* red) {
    const int lane = threadIdx.x & (kWave - 1);
    const int b = blk * int(blockDim.x / kWave) + int(threadIdx.x / kWave);
    double acc[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[k] = 0.0;
    if (b < L.B) {
        for (int t = lane; t < L.T; t += kWave) {
            const float* rec = L.ws.tokrec + (int64_t(b) * L.T + t) * kTokRec;
            float f[11];
#pragma unroll
            for (int k = 0; k < 11; ++k) f[k] = rec[k];
            acc[0] += double(f[0]);
            acc[1] += double(f[1]);
            acc[2] += double(f[2]);
            acc[3] += double(f[3]);
            acc[4] += double(f[4]);
            acc[5] += double(f[5]);
            acc[6] += double(f[5]) * double(f[5]);
            acc[7] += double(f[6]);
            acc[8] += double(f[7]);
            acc[9] += double(f[8]);
            acc[10] += double(f[8]) * double(f[8]);
            acc[11] += double(f[9]);
            acc[12] += double(f[10]);
        }
    }
    const double rec = block_sum_multi<16>(acc, red);
    if (publish_record_last<16>(L.ws.loss_rec + blk * 16, rec, L.ws.tickets + 1, unsigned(nblk))) {
        __syncthreads();  // red[] reuse
        const double tot = reduce_records<16>(L.ws.loss_rec, nblk, red);
        __syncthreads();
        if (threadIdx.x < 16) red[threadIdx.x] = tot;
        __syncthreads();
        if (threadIdx.x == 0) {
            double a[kLossSums];
            for (int k = 0; k < kLossSums; ++k) a[k] = red[k];
            const double msum = L.msum ? *L.msum : double(int64_t(L.B) * L.T);
            float s13[TRLX_PPO_STATS];
            emit_loss_stats(a, double(int64_t(L.B) * L.T), msum, L.vf_coef, L.loss, s13);
            for (int k = 0; k < TRLX_PPO_STATS; ++k) L.stats[k] = s13[k];
            kl_ctl_apply(L.kl, s13[8]);  // policy/approx_kl
        }
    }
}

#ifndef TRLX_ROW_TAILS_NO_KERNELS
__global__ __launch_bounds__(kRolloutThreads) void k_rollout_loss(LossRolloutArgs L) {
    __shared__ double red[kRolloutsPerBlock * 16];
    loss_tail_block(L, int(blockIdx.x), int(gridDim.x), red);
}
#endif

}  // namespace trlx
