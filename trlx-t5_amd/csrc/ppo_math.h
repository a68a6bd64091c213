// Per-token PPO arithmetic shared by the fused vocab-row kernel and the [B,T] loss kernel.
#pragma once
#include "common.h"

namespace trlx {

// Closed-form d(policy loss)/d(logprob) for one token, following the autograd graph of
// ppo_models.py:165-177:  lr = (lp-olp)*m;  ratio = exp(lr);
//   pg = max(-A*ratio, -A*clamp(ratio, 1-c, 1+c));  loss_pg = sum(pg*m) / sum(m)
// torch.maximum splits the gradient 1/2-1/2 on ties; clamp passes it on its inclusive
// bounds.  Also returns the forward terms the stats need.
struct PolicyTerms {
    float ratio, lr, pgmax;
    bool pgclip;
};
__device__ __forceinline__ float ppo_policy_dlp(float lp, float olp, float A, float m, float inv_msum,
                                                float c, PolicyTerms& o) {
    o.lr = mul_rn(lp - olp, m);
    o.ratio = expf(o.lr);
    const float negA = -A;
    const float lo = 1.0f - c, hi = 1.0f + c;
    const float pg1 = mul_rn(negA, o.ratio);
    const float cr = fminf(fmaxf(o.ratio, lo), hi);
    const float pg2 = mul_rn(negA, cr);
    o.pgmax = fmaxf(pg1, pg2);
    o.pgclip = pg2 > pg1;
    const float u = mul_rn(inv_msum, m);
    float g1, g2;
    if (pg1 == pg2) {
        g1 = u * 0.5f;
        g2 = g1;
    } else {
        g1 = pg1 > pg2 ? u : 0.0f;
        g2 = pg1 > pg2 ? 0.0f : u;
    }
    const float inr = (o.ratio >= lo && o.ratio <= hi) ? 1.0f : 0.0f;
    const float dratio = add_rn(mul_rn(g1, negA), mul_rn(mul_rn(g2, negA), inr));
    return mul_rn(mul_rn(dratio, o.ratio), m);
}

// mean and rsqrt(var + 1e-8) from a {sum, sumsq, count} fp64 record (modeling.py:24-34):
// var = M2/count in the distributed branch, M2/(count-1) for torch.var_mean.
// No fp64 division (its v_div_scale/v_rcp sequence would set the fused row kernel's
// register peak): 1/n is the fp32 reciprocal refined by two Newton steps in fp64 (exact to
// ~1 ulp of a double), so mu = fl32(Σx · 1/n) is the correctly rounded mean (torch's fp32
// mean of an fp64 accumulation) even at a large common offset, where rounding Σx to fp32
// first could move mu by an ulp (1e-3 at |mu| ~ 1e4: every whitened value would shift by
// it).  M2 = Σx² − 2·m·Σx + n·m² with m = the fp32 mean is exact up to n·(μ − m)² (~1e-14
// relative), evaluated with fp64 fmas.
__device__ __forceinline__ void whiten_coeffs(const double* st, int unbiased, float& mu, float& rstd) {
    const double sum = st[0], sumsq = st[1], cnt = st[2];
    const float nf = float(cnt);
    double r = double(__frcp_rn(nf));
    r = r * fma(-cnt, r, 2.0);
    r = r * fma(-cnt, r, 2.0);
    mu = float(sum * r);
    const double m = double(mu);
    double m2 = fma(m * cnt, m, fma(-2.0 * m, sum, sumsq));
    if (m2 < 0) m2 = 0;
    rstd = rsqrtf(float(m2) / (unbiased ? nf - 1.0f : nf) + 1e-8f);
}

// Loss and the 13 stats of PPOConfig.loss (ppo_models.py:162-198) from fp64 sums:
//   acc[0] Σ max(vl1,vl2)·m   acc[1] #(vl2 > vl1)   acc[2] Σ (ratio-1) - log_ratio
//   acc[3] Σ max(pg1,pg2)·m   acc[4] #(pg2 > pg1)   acc[5] Σ old_values   acc[6] Σ old_values²
//   acc[7] Σ values           acc[8] Σ (values-returns)²                  acc[9] Σ returns
//   acc[10] Σ returns²        acc[11] Σ ratio·m     acc[12] Σ m
// Divisions by N are torch.mean; var is torch.var (unbiased).
constexpr int kLossSums = 13;
__device__ __forceinline__ void emit_loss_stats(const double* acc, double N, double msum, float vf_coef,
                                                float* loss, float* s) {
    const double vf = 0.5 * acc[0] / msum;
    const double pg = acc[3] / msum;
    const double tot = pg + double(vf_coef) * vf;
    loss[0] = float(tot);
    s[0] = float(tot);                                         // losses/total_loss
    s[1] = float(pg);                                          // losses/policy_loss
    s[2] = float(vf);                                          // losses/value_loss
    s[3] = float(acc[5] / N);                                  // values/mean_old_values
    s[4] = float((acc[6] - acc[5] * acc[5] / N) / (N - 1.0));  // values/var_old_values
    s[5] = float(acc[7] / N);                                  // values/mean_values
    s[6] = float(acc[8] / N);                                  // values/values_error
    s[7] = float(acc[1] / N);                                  // values/clipfrac
    s[8] = float(acc[2] / N);                                  // policy/approx_kl
    s[9] = float(acc[4] / N);                                  // policy/clipfrac
    s[10] = float(acc[9] / N);                                 // returns/mean
    s[11] = float((acc[10] - acc[9] * acc[9] / N) / (N - 1.0));  // returns/var
    s[12] = float(acc[11] / msum);                             // ratio
}

}  // namespace trlx
