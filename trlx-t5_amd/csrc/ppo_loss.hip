// PPOConfig.loss (trlx/model/nn/ppo_models.py:141-199) over [B,T] per-token vectors:
// a grid-stride elementwise pass that writes the per-token gradients and fp64 partial
// sums, then a single-block fixed-order finalize that produces the loss and the 13
// stats.  Deterministic (no atomics).
#include "ppo_math.h"

namespace trlx {

struct LossArgs {
    int64_t n;
    const void* lp; int lp_dtype;
    const void* v; int v_dtype;
    const void* olp; int olp_dtype;
    const void* ov; int ov_dtype;
    const void* adv; int a_dtype;
    const double* adv_stats; int unbiased;
    const void* ret; int r_dtype;
    const int64_t* mask;
    const double* msum; double msum_host;
    float c, cv, vf_coef;
    void* dlp; void* dv; int g_dtype;
    double* partials;
    float* loss; float* stats; unsigned* ticket;  // optional fused finalize (last block)
};

constexpr int kLossThreads = 256;
constexpr int kLossPerBlock = kLossThreads * 2;  // many short blocks: latency, not bandwidth, bound
constexpr int kSlots = TRLX_PPO_PARTIAL_SLOTS;

// Loss and the 13 stats from the fixed-order totals of the records (ppo_models.py:162-198;
// the divisions by N are torch.mean, var is unbiased).  `tot` lives in threads k < kSlots
// (block_sum_multi layout); thread 0 gathers them through `sh`.
__device__ void ppo_loss_emit(double tot, int64_t n, double msum, float vf_coef, float* loss, float* stats,
                              double* sh) {
    __syncthreads();
    if (threadIdx.x < kSlots) sh[threadIdx.x] = tot;
    __syncthreads();
    if (threadIdx.x != 0) return;
    double acc[kSlots];
    for (int k = 0; k < kSlots; ++k) acc[k] = sh[k];
    emit_loss_stats(acc, double(n), msum, vf_coef, loss, stats);
}

__global__ __launch_bounds__(kLossThreads) void k_ppo_loss_elem(LossArgs a) {
    __shared__ double red[(kLossThreads / kWave) * kSlots];
    const int64_t beg = int64_t(blockIdx.x) * kLossPerBlock;
    const int64_t end = min<int64_t>(a.n, beg + kLossPerBlock);
    float mu = 0.f, rstd = 1.f;
    if (a.adv_stats) whiten_coeffs(a.adv_stats, a.unbiased, mu, rstd);
    const double msum = a.msum ? *a.msum : a.msum_host;
    const float inv_msum = 1.0f / float(msum);
    // d loss / d vf = vf_coef; vf = (0.5 * sum(max(vl1,vl2)*m)) / msum
    const float uv = mul_rn(a.vf_coef / float(msum), 0.5f);
    double acc[kSlots];
#pragma unroll
    for (int k = 0; k < kSlots; ++k) acc[k] = 0.0;

    for (int64_t i = beg + threadIdx.x; i < end; i += kLossThreads) {
        const float lp = ld_any(a.lp, a.lp_dtype, i);
        const float v = ld_any(a.v, a.v_dtype, i);
        const float olp = ld_any(a.olp, a.olp_dtype, i);
        const float ov = ld_any(a.ov, a.ov_dtype, i);
        float A = ld_any(a.adv, a.a_dtype, i);
        if (a.adv_stats) A = mul_rn(A - mu, rstd);
        const float R = ld_any(a.ret, a.r_dtype, i);
        const float m = a.mask ? float(a.mask[i]) : 1.0f;
        // value loss (ppo_models.py:155-163)
        const float vlo = ov - a.cv, vhi = ov + a.cv;
        const float vc = fminf(fmaxf(v, vlo), vhi);
        const float e1 = v - R, e2 = vc - R;
        const float vl1 = mul_rn(e1, e1), vl2 = mul_rn(e2, e2);
        const float vmax = fmaxf(vl1, vl2);
        // policy loss (ppo_models.py:165-178)
        PolicyTerms pt;
        const float g = ppo_policy_dlp(lp, olp, A, m, inv_msum, a.c, pt);
        if (a.dlp) st_any(a.dlp, a.g_dtype, i, g);
        if (a.dv) {
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
            const float d1 = mul_rn(mul_rn(h1, 2.0f), e1);
            const float d2 = mul_rn(mul_rn(mul_rn(h2, 2.0f), e2), inr);
            st_any(a.dv, a.g_dtype, i, add_rn(d1, d2));
        }
        acc[0] += double(mul_rn(vmax, m));
        acc[1] += vl2 > vl1 ? 1.0 : 0.0;
        acc[2] += double((pt.ratio - 1.0f) - pt.lr);
        acc[3] += double(mul_rn(pt.pgmax, m));
        acc[4] += pt.pgclip ? 1.0 : 0.0;
        acc[5] += double(ov);
        acc[6] += double(ov) * double(ov);
        acc[7] += double(v);
        acc[8] += double(vl1);
        acc[9] += double(R);
        acc[10] += double(R) * double(R);
        acc[11] += double(mul_rn(pt.ratio, m));
        acc[12] += double(m);
    }
    const double rec = block_sum_multi<kSlots>(acc, red);
    double* my = a.partials + blockIdx.x * kSlots;
    if (!a.ticket) {
        if (threadIdx.x < kSlots) my[threadIdx.x] = rec;
        return;
    }
    if (publish_record_last<kSlots>(my, rec, a.ticket, gridDim.x)) {
        __syncthreads();  // red[] reuse
        const double tot = reduce_records<kSlots>(a.partials, gridDim.x, red);
        ppo_loss_emit(tot, a.n, msum, a.vf_coef, a.loss, a.stats, red);
    }
}

__global__ __launch_bounds__(256) void k_ppo_loss_finalize(const double* partials, int64_t nblk, int64_t n,
                                                           const double* msum_p, double msum_host,
                                                           float vf_coef, float* loss, float* stats) {
    __shared__ double red[(256 / kWave) * kSlots];
    const double tot = reduce_records<kSlots>(partials, int(nblk), red);
    ppo_loss_emit(tot, n, msum_p ? *msum_p : msum_host, vf_coef, loss, stats, red);
}

// ------------------------------------------------------------------ autograd scaling
// out = x * (*scale).  In place (out == x) the launch is a no-op when *scale == 1, the
// common loss.backward() case, so the fused dlogits cost no extra pass.
__global__ void k_scale_by(const void* x, void* out, int dtype, int64_t n, const float* scale) {
    const float s = *scale;
    if (s == 1.0f && x == out) return;
    for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n;
         i += int64_t(gridDim.x) * blockDim.x)
        st_any(out, dtype, i, ld_any(x, dtype, i) * s);
}

}  // namespace trlx

using namespace trlx;

extern "C" int64_t trlx_ppo_loss_num_blocks(int64_t n) {
    return n <= 0 ? 1 : (n + kLossPerBlock - 1) / kLossPerBlock;
}

extern "C" int trlx_ppo_loss_elem(int64_t n, const void* lp, int lp_dtype, const void* values, int v_dtype,
                                  const void* old_lp, int olp_dtype, const void* old_values, int ov_dtype,
                                  const void* adv, int a_dtype,
                                  const double* adv_stats, int unbiased, const void* returns, int r_dtype,
                                  const int64_t* mask, const double* msum, double msum_host,
                                  float cliprange, float cliprange_value, float vf_coef, void* dlp,
                                  void* dv, int g_dtype, double* partials, float* loss, float* stats,
                                  unsigned* ticket, void* stream) {
    TRLX_REQUIRE(lp && values && old_lp && old_values && adv && returns && partials, TRLX_ERR_ARG,
                 "NULL input to ppo loss");
    TRLX_REQUIRE(msum || msum_host > 0, TRLX_ERR_ARG, "mask sum must be positive");
    TRLX_REQUIRE(n > 0, TRLX_ERR_SHAPE, "empty loss input");
    LossArgs a = {};
    a.n = n; a.lp = lp; a.lp_dtype = lp_dtype; a.v = values; a.v_dtype = v_dtype; a.olp = old_lp; a.olp_dtype = olp_dtype;
    a.ov = old_values; a.ov_dtype = ov_dtype; a.adv = adv; a.a_dtype = a_dtype; a.adv_stats = adv_stats; a.unbiased = unbiased;
    a.ret = returns; a.r_dtype = r_dtype; a.mask = mask; a.msum = msum; a.msum_host = msum_host;
    a.c = cliprange; a.cv = cliprange_value; a.vf_coef = vf_coef; a.dlp = dlp; a.dv = dv;
    a.g_dtype = g_dtype; a.partials = partials; a.loss = loss; a.stats = stats; a.ticket = ticket;
    TRLX_REQUIRE(!ticket || (loss && stats), TRLX_ERR_ARG, "fused finalize needs loss and stats");
    hipLaunchKernelGGL(k_ppo_loss_elem, dim3(unsigned(trlx_ppo_loss_num_blocks(n))), dim3(kLossThreads), 0,
                       (hipStream_t)stream, a);
    return check_launch("k_ppo_loss_elem");
}

extern "C" int trlx_ppo_loss_finalize(const double* partials, int64_t nblk, int64_t n, const double* msum,
                                      double msum_host, float vf_coef, float* loss, float* stats,
                                      void* stream) {
    TRLX_REQUIRE(partials && loss && stats && nblk > 0, TRLX_ERR_ARG, "bad finalize args");
    hipLaunchKernelGGL(k_ppo_loss_finalize, dim3(1), dim3(256), 0, (hipStream_t)stream, partials, nblk, n,
                       msum, msum_host, vf_coef, loss, stats);
    return check_launch("k_ppo_loss_finalize");
}

extern "C" int trlx_scale_by(const void* x, void* out, int dtype, int64_t n, const float* scale,
                             void* stream) {
    TRLX_REQUIRE(x && out && scale, TRLX_ERR_ARG, "NULL x/out/scale");
    if (n == 0) return TRLX_OK;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(k_scale_by, dim3(unsigned(blocks)), dim3(256), 0, (hipStream_t)stream, x, out, dtype, n,
                       scale);
    return check_launch("k_scale_by");
}
