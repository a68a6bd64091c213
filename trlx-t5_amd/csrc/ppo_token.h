// Per-token arithmetic of the fused PPO loss shared by the vocab-row kernels (vocab_rows.hip,
// which read each token's logits row) and the fused lm_head loss (lmhead_loss.hip, which never
// materialises it): the token's whitened advantage, mask and normaliser (ppo_scalars), the
// split-beta reward / return outputs, and the loss record the loss tail sums (row_tails.h).
// Templated over the launch's argument struct: every field used here has the same name in
// RowArgs and LmLossArgs.
#pragma once
#include "row_tails.h"

namespace trlx {

// The PPO workspace carve-up (tickets, GAE / loss block records, token records, row order):
// vocab_rows.hip; the fused lm_head loss writes the same token records.
size_t carve_ppo_workspace(void* base, int64_t B, int64_t T, Workspace* w);

// Row-independent per-token scalars of the fused PPO mode.  Split-beta rows only: beta, the
// coefficients, and the token's reward and return (ppo_orchestrator.py:164-167,
// ppo_models.py:135), stored by split_outputs after the row.
struct PpoScalars {
    float A, m, inv_msum, olp;
    float beta, mu, rstd, rew, R;
};
// Split beta: the token's value-loss inputs {values, old_values, returns}, the return A + V
// finished here from A = A0 - beta*Ak (R: as computed; vin[2]: as stored, which the value
// loss sees).  No stores here: a store ahead of the row's loads would hold them back (the
// buffer loads may not move above it).
template <class Args>
__device__ __forceinline__ void split_value_inputs(const Args& a, int64_t row, float A, float* vin, float& R) {
    vin[0] = ld_any(a.ltok.values, a.ltok.v_dtype, row);
    vin[1] = ld_any(a.ltok.old_values, a.ltok.ov_dtype, row);
    R = add_rn(A, vin[1]);
    vin[2] = a.ltok.r_dtype == TRLX_BF16 ? bf2f(f2bf(R)) : R;
}
// After the row (thread 0): the split-beta token outputs — reward, return, and (row 0) the
// whitening coefficients the rows derived, for a later loss on the same experience.
template <class Args>
__device__ __forceinline__ void split_outputs(const Args& a, int64_t row, const PpoScalars& p) {
    a.rewards_out[row] = p.rew;
    st_any(const_cast<void*>(a.ltok.returns), a.ltok.r_dtype, row, p.R);
    if (row == 0 && a.coef_out) {
        a.coef_out[0] = p.mu;
        a.coef_out[1] = p.rstd;
        a.coef_out[2] = p.beta;
        a.coef_out[3] = 0.0f;
    }
}
template <class Args>
__device__ __forceinline__ float split_advantage(const Args& a, int64_t row, float beta) {
    return a.adv[row] - mul_rn(beta, a.adv_kl[row]);
}
// The split-beta whitening coefficients {mu, rstd, beta} of this launch: derived from the
// batch's record (wstats; row 0 publishes them in split_outputs) or read from a coef vector.
template <class Args>
__device__ __forceinline__ void split_coef(const Args& a, int64_t row, float& mu, float& rstd, float& beta) {
    if (a.wstats) {
        beta = a.wctl ? float(a.wctl[TRLX_CTL_KL_COEF]) : a.wbeta;
        whiten_split_coeffs(a.wstats, a.wunbiased, beta, mu, rstd);
    } else {
        mu = a.coef[0];
        rstd = a.coef[1];
        beta = a.coef[2];
    }
}

// vin (fused loss, tokrec set): {values, old_values, returns} of the token's value loss,
// loaded here when `early` (the resident rows park them in LDS; the streaming rows load
// them after the row).
template <class Args>
__device__ __forceinline__ PpoScalars ppo_scalars(const Args& a, int64_t row, float* vin, bool early) {
    PpoScalars p;
    p.A = a.adv[row];
    p.beta = p.mu = p.rstd = p.rew = p.R = 0.0f;
    if (a.coef || a.wstats) {  // split beta: this token's advantage, reward and return are finished here
        split_coef(a, row, p.mu, p.rstd, p.beta);
        const float A = split_advantage(a, row, p.beta);
        p.rew = add_rn(mul_rn(-p.beta, a.rew_kl[row]), a.rew_score[row]);
        p.A = mul_rn(A - p.mu, p.rstd);
        if (early && a.tokrec) split_value_inputs(a, row, A, vin, p.R);
    } else if (a.stats) {
        float mu, rstd;
        whiten_coeffs(a.stats, a.unbiased, mu, rstd);
        p.A = mul_rn(p.A - mu, rstd);
        if (early && a.tokrec) loss_token_inputs(a.ltok, row, vin);
    } else if (early && a.tokrec) {
        loss_token_inputs(a.ltok, row, vin);
    }
    p.m = a.mask ? float(a.mask[row]) : 1.0f;
    const double msum = a.msum ? *a.msum : a.msum_host;
    p.inv_msum = 1.0f / float(msum);  // torch: grad / mask.sum()
    p.olp = ld_any(a.old_lp, a.old_dtype, row);
    return p;
}

// After the row is stored (its registers dead): the token's loss record (fused loss);
// vin = {values, old_values, returns} loaded in the prologue (loss_token_inputs).
template <class Args>
__device__ __forceinline__ void token_record(const Args& a, int64_t row, const PolicyTerms& pt,
                                             const PpoScalars& ps, const float* vin) {
    if (a.tokrec && threadIdx.x == 0)
        loss_token_terms(a.ltok, a.tokrec, row, pt, ps.m, ps.inv_msum, vin[0], vin[1], vin[2]);
}

}  // namespace trlx
