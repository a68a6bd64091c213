// Work hidden in the tails of the vocab-row kernels.
//
// Every token row is one workgroup.  When the last of a rollout's row-workgroups
// finishes (per-rollout arrival ticket), that workgroup runs the rollout's [T]-vector
// work — the GAE scan after the experience rows, the per-token loss terms' sum after
// the fused loss rows — and publishes one fp64 record; the last rollout to finish
// (global ticket) reduces the records.  The whole experience+loss step is then two
// launches, and the O(B*T) work overlaps the O(B*T*V) streaming of other rows.
//
// Cross-workgroup hand-off: fence-free write-through form (MI355X_MICROARCH.md "Valid
// forms", row 1): payload stored `sc1` by the storing wave, drained with
// `s_waitcnt vmcnt(0)`, then ONE lane's agent-scope atomic add; the workgroup whose add
// returns count-1 reads the payload with `sc1` loads.  Every payload line is read once,
// after its last write, inside the launch.  Tickets are zero at launch and re-armed by
// their last arrival.
#pragma once
#include "ppo_math.h"

namespace trlx {

constexpr int kAuxSC1 = 16;  // buffer-op aux: sc1 (write-through store / L1-bypassing load)

__device__ __forceinline__ void st_sc1(float* p, float v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Called by ONE lane after its sc1 payload stores: drain, arrive, return the old count.
// Re-arms the ticket when this arrival completes the group of `group` arrivals.
__device__ __forceinline__ bool arrive_last(unsigned* ticket, unsigned group) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool last = (t == group - 1);
    if (last) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return last;
}

// Wave-wide fixed-order (butterfly) sum; every lane ends with the total.
__device__ __forceinline__ double wave_allsum_d(double v) {
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) v += __shfl_xor(v, off, kWave);
    return v;
}

// ------------------------------------------------------------------ experience tail
// Workspace layout (bytes, 16-B aligned sections), see trlx_ppo_workspace_bytes:
//   tickets  : uint32[B] per-rollout + uint32 global (+pad)      (must start zeroed)
//   records  : double[B][4]   per-rollout {Σ A, Σ A², n, Σ mask}
//   tokrec   : float[B*T][16] per-token loss terms (loss tail)
//   rowrec   : double[B][16]  per-rollout loss sums (loss tail)
struct Workspace {
    unsigned* row_ticket;  // [B]
    unsigned* all_ticket;  // [1]
    double* mom;           // [B][4]
    float* tokrec;         // [B*T][16]
    double* rowrec;        // [B][16]
    unsigned* row_ticket2; // [B]   (loss tail)
    unsigned* all_ticket2; // [1]
};

struct ExpTailArgs {
    const void* values;   // [B,T] old values (the experience forward's values)
    int v_dtype;
    const float* scores;  // [B] or NULL
    const int64_t* lengths;  // [B] or NULL
    const int64_t* mask;     // [B,T] loss mask or NULL
    float neg_beta, gamma, gl;
    float* rewards;       // [B,T] fp32 out
    float* adv;           // [B,T] fp32 out (unwhitened)
    void* ret;            // [B,T] out
    int ret_dtype;
    double* stats;        // [4] out: Σ A, Σ A², n, Σ mask
};

// GAE for rollout b by wave 0 of the workgroup that completed the rollout's rows.
// Suffix recurrence A_t = δ_t + c·A_{t+1} as a lane-parallel scan (log2 64 steps) over
// 64-token chunks from the end, with the chunk carry A_{chunk end} weighted c^(n).
// (fp32 re-association vs the reference's sequential loop: ~1e-7 relative.)
__device__ void experience_tail_row(const ExpTailArgs& e, const Workspace& w, int b, int T,
                                    const float* lp, const float* ref_lp, int B) {
    const int lane = threadIdx.x;  // wave 0 only
    const int len = e.lengths ? int(e.lengths[b]) : T;
    const float log2c = e.gl > 0.0f ? __log2f(e.gl) : -INFINITY;
    float carry = 0.0f, vcarry = 0.0f;  // A and V just past the current chunk
    double s1 = 0.0, s2 = 0.0, sm = 0.0;
    for (int c0 = ((T - 1) / kWave) * kWave; c0 >= 0; c0 -= kWave) {
        const int t = c0 + lane;
        const bool ok = t < T;
        const int64_t gi = int64_t(b) * T + t;
        float v = 0.0f, r = 0.0f;
        if (ok && t < len) {
            v = ld_any(e.values, e.v_dtype, gi);
            r = mul_rn(e.neg_beta, ld_sc1(lp + gi) - ld_sc1(ref_lp + gi));
            if (t == len - 1 && e.scores) r = add_rn(r, e.scores[b]);
        }
        float vn = __shfl_down(v, 1, kWave);
        if (lane == kWave - 1) vn = vcarry;
        const float delta = ok ? add_rn(r, mul_rn(e.gamma, vn)) - v : 0.0f;
        // lane-parallel suffix scan inside the chunk
        float x = delta, cd = e.gl;
#pragma unroll
        for (int d = 1; d < kWave; d <<= 1) {
            const float y = __shfl_down(x, d, kWave);
            if (lane + d < kWave) x = fmaf(cd, y, x);
            cd = cd * cd;
        }
        const int end = min(c0 + kWave, T);
        const float A = ok ? fmaf(exp2_fast(float(end - t) * log2c), carry, x) : 0.0f;
        carry = __shfl(A, 0, kWave);
        vcarry = __shfl(v, 0, kWave);
        if (ok) {
            e.rewards[gi] = r;
            e.adv[gi] = A;
            st_any(e.ret, e.ret_dtype, gi, add_rn(A, v));
            s1 += double(A);
            s2 += double(A) * double(A);
            sm += e.mask ? double(e.mask[gi]) : 1.0;
        }
    }
    s1 = wave_allsum_d(s1);
    s2 = wave_allsum_d(s2);
    sm = wave_allsum_d(sm);
    bool last = false;
    if (lane == 0) {
        double* rec = w.mom + b * 4;
        st_sc1(rec + 0, s1);
        st_sc1(rec + 1, s2);
        st_sc1(rec + 2, double(T));
        st_sc1(rec + 3, sm);
        last = arrive_last(w.all_ticket, unsigned(B));
    }
    last = __shfl(last ? 1 : 0, 0, kWave) != 0;
    if (!last) return;
    // the last rollout: fixed-order reduction of the B records
    double a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    for (int i = lane; i < B; i += kWave) {
        const double* rec = w.mom + i * 4;
        a0 += ld_sc1(rec + 0);
        a1 += ld_sc1(rec + 1);
        a2 += ld_sc1(rec + 2);
        a3 += ld_sc1(rec + 3);
    }
    a0 = wave_allsum_d(a0);
    a1 = wave_allsum_d(a1);
    a2 = wave_allsum_d(a2);
    a3 = wave_allsum_d(a3);
    if (lane == 0) {
        e.stats[0] = a0;
        e.stats[1] = a1;
        e.stats[2] = a2;
        e.stats[3] = a3;
    }
}

// ------------------------------------------------------------------ loss tail
constexpr int kTokRec = 16;  // floats per token record (13 used)

struct LossTailArgs {
    const void* values;      // [B,T] new values (requires grad in the reference)
    int v_dtype;
    const void* old_values;  // [B,T]
    int ov_dtype;
    const void* returns;     // [B,T]
    int r_dtype;
    float cv, vf_coef;
    float* dv;               // [B,T] fp32 out: d loss / d values
    float* loss;             // [1] out
    float* stats;            // [13] out
};

// Per-token terms of PPOConfig.loss (ppo_models.py:155-178) for token `row`, stored as a
// write-through record; also writes d loss / d values.  Thread 0 only.
__device__ void loss_token_terms(const LossTailArgs& L, const Workspace& w, int64_t row, float lp_unused,
                                 const PolicyTerms& pt, float m, float inv_msum) {
    (void)lp_unused;
    const float v = ld_any(L.values, L.v_dtype, row);
    const float ov = ld_any(L.old_values, L.ov_dtype, row);
    const float R = ld_any(L.returns, L.r_dtype, row);
    const float vlo = ov - L.cv, vhi = ov + L.cv;
    const float vc = fminf(fmaxf(v, vlo), vhi);
    const float e1 = v - R, e2 = vc - R;
    const float vl1 = mul_rn(e1, e1), vl2 = mul_rn(e2, e2);
    // d loss / d v (value term, same tie / bound rules as the policy term)
    const float uv = mul_rn(mul_rn(L.vf_coef, inv_msum), 0.5f);
    const float u = mul_rn(uv, m);
    float h1, h2;
    if (vl1 == vl2) {
        h1 = u * 0.5f;
        h2 = h1;
    } else {
        h1 = vl1 > vl2 ? u : 0.0f;
        h2 = vl1 > vl2 ? 0.0f : u;
    }
    const float inr = (v >= vlo && v <= vhi) ? 1.0f : 0.0f;
    L.dv[row] = add_rn(mul_rn(mul_rn(h1, 2.0f), e1), mul_rn(mul_rn(mul_rn(h2, 2.0f), e2), inr));
    float* rec = w.tokrec + row * kTokRec;
    st_sc1(rec + 0, mul_rn(fmaxf(vl1, vl2), m));
    st_sc1(rec + 1, vl2 > vl1 ? 1.0f : 0.0f);
    st_sc1(rec + 2, (pt.ratio - 1.0f) - pt.lr);
    st_sc1(rec + 3, mul_rn(pt.pgmax, m));
    st_sc1(rec + 4, pt.pgclip ? 1.0f : 0.0f);
    st_sc1(rec + 5, ov);
    st_sc1(rec + 6, v);
    st_sc1(rec + 7, vl1);
    st_sc1(rec + 8, R);
    st_sc1(rec + 9, mul_rn(pt.ratio, m));
    st_sc1(rec + 10, m);
}

constexpr int kLossSums = 13;  // fp64 per-rollout sums (see loss_tail_row)

// Wave 0 of the workgroup that completed rollout b's rows: sum its T token records in
// fp64 (sums and sums of squares), publish; the last rollout emits loss + 13 stats.
__device__ void loss_tail_row(const LossTailArgs& L, const Workspace& w, int b, int T, int B, double msum) {
    const int lane = threadIdx.x;
    double acc[kLossSums];
#pragma unroll
    for (int k = 0; k < kLossSums; ++k) acc[k] = 0.0;
    for (int t = lane; t < T; t += kWave) {
        const float* rec = w.tokrec + (int64_t(b) * T + t) * kTokRec;
        float f[11];
#pragma unroll
        for (int k = 0; k < 11; ++k) f[k] = ld_sc1(rec + k);
        acc[0] += double(f[0]);                    // Σ max(vl1,vl2)·m
        acc[1] += double(f[1]);                    // vf clip count
        acc[2] += double(f[2]);                    // Σ (ratio-1) - log_ratio
        acc[3] += double(f[3]);                    // Σ max(pg1,pg2)·m
        acc[4] += double(f[4]);                    // pg clip count
        acc[5] += double(f[5]);                    // Σ old_values
        acc[6] += double(f[5]) * double(f[5]);     // Σ old_values²
        acc[7] += double(f[6]);                    // Σ values
        acc[8] += double(f[7]);                    // Σ (values - returns)²
        acc[9] += double(f[8]);                    // Σ returns
        acc[10] += double(f[8]) * double(f[8]);    // Σ returns²
        acc[11] += double(f[9]);                   // Σ ratio·m
        acc[12] += double(f[10]);                  // Σ m
    }
#pragma unroll
    for (int k = 0; k < kLossSums; ++k) acc[k] = wave_allsum_d(acc[k]);
    bool last = false;
    if (lane == 0) {
        double* rec = w.rowrec + int64_t(b) * 16;
#pragma unroll
        for (int k = 0; k < kLossSums; ++k) st_sc1(rec + k, acc[k]);
        last = arrive_last(w.all_ticket2, unsigned(B));
    }
    last = __shfl(last ? 1 : 0, 0, kWave) != 0;
    if (!last) return;
#pragma unroll
    for (int k = 0; k < kLossSums; ++k) acc[k] = 0.0;
    for (int i = lane; i < B; i += kWave) {
        const double* rec = w.rowrec + int64_t(i) * 16;
#pragma unroll
        for (int k = 0; k < kLossSums; ++k) acc[k] += ld_sc1(rec + k);
    }
#pragma unroll
    for (int k = 0; k < kLossSums; ++k) acc[k] = wave_allsum_d(acc[k]);
    if (lane != 0) return;
    const double N = double(int64_t(B) * T);
    const double vf = 0.5 * acc[0] / msum;
    const double pg = acc[3] / msum;
    const double tot = pg + double(L.vf_coef) * vf;
    L.loss[0] = float(tot);
    float* s = L.stats;
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
