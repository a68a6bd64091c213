// [B, T] per-token kernels: KL-penalised reward, GAE reverse scan (+ fused KL reward,
// + whitening partial moments), batch moments / whitening.
//
// These move O(B*T) bytes (tens of KB .. MB) and are latency-bound, not bandwidth-bound:
// the design goal is few launches and a deterministic fixed-order fp64 reduction, not
// peak GB/s.
#include "common.h"

namespace trlx {

// ------------------------------------------------------------------ A2
// ppo_orchestrator.py:164-167: kls = lp - ref_lp; r = -beta*kls; r[:, -1] += score
__device__ __forceinline__ float kl_reward(float lp, float ref_lp, float neg_beta, int64_t t,
                                           int64_t last, const float* scores, int64_t b) {
    float r = mul_rn(neg_beta, lp - ref_lp);
    if (t == last && scores) r = add_rn(r, scores[b]);
    return r;
}

__global__ void k_kl_rewards(const void* lp, const void* ref_lp, int in_dtype, int64_t B, int64_t T,
                             float neg_beta, const float* scores, const int64_t* lengths,
                             void* out, int out_dtype) {
    const int64_t n = B * T;
    for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n;
         i += int64_t(gridDim.x) * blockDim.x) {
        const int64_t b = i / T, t = i - (i / T) * T;
        const int64_t len = lengths ? lengths[b] : T;
        float r = 0.0f;
        if (t < len)
            r = kl_reward(ld_any(lp, in_dtype, i), ld_any(ref_lp, in_dtype, i), neg_beta, t, len - 1,
                          scores, b);
        st_any(out, out_dtype, i, r);
    }
}

// ------------------------------------------------------------------ A5
struct GaeArgs {
    const void* values;
    const void* rewards;
    int dtype;
    int B, T, Teff;
    float gamma, gl;  // gamma, gamma*lam (rounded to fp32 like the torch scalar)
    const float* lp;
    const float* ref_lp;
    float neg_beta;
    const float* scores;
    const int64_t* lengths;
    const int64_t* mask;
    float* adv;
    void* ret;
    int ret_dtype;
    void* rew_out;
    int rew_dtype;
    double* partials;
    double* stats;       // optional: last block reduces the partials into stats[4]
    unsigned* ticket;    // required with stats
    int rpb;     // rows per block
    int stride;  // LDS row stride (odd => conflict-free column walk)
};

constexpr int kGaeThreads = 256;
constexpr int kGaeMaxRows = 16;      // rows per block: many small blocks, short staging loops
constexpr int kGaeLdsFloats = 8192;  // per array (32 KB)

__global__ __launch_bounds__(kGaeThreads) void k_gae(GaeArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    __shared__ double red[(kGaeThreads / kWave) * TRLX_MOMENT_SLOTS];
    float* sv = lds;                        // values, then returns
    float* sr = lds + a.rpb * a.stride;     // rewards, then advantages
    const int tid = threadIdx.x;
    const int row0 = blockIdx.x * a.rpb;
    const int rows = min(a.rpb, a.B - row0);
    const int nel = rows * a.Teff;

    // ---- stage values / rewards (coalesced: rows are contiguous with stride T)
    double msum = 0.0;
    for (int e = tid; e < nel; e += kGaeThreads) {
        const int r = e / a.Teff;
        const int c = e - r * a.Teff;
        const int b = row0 + r;
        const int64_t gi = int64_t(b) * a.T + c;
        const int len = a.lengths ? int(a.lengths[b]) : a.T;
        float v = 0.0f, rw = 0.0f;
        if (c < len) {
            v = ld_any(a.values, a.dtype, gi);
            rw = a.lp ? kl_reward(a.lp[gi], a.ref_lp[gi], a.neg_beta, c, len - 1, a.scores, b)
                      : ld_any(a.rewards, a.dtype, gi);
        }
        if (a.lp && a.rew_out) st_any(a.rew_out, a.rew_dtype, gi, rw);
        sv[r * a.stride + c] = v;
        sr[r * a.stride + c] = rw;
        msum += a.mask ? double(a.mask[int64_t(b) * a.Teff + c]) : 1.0;
    }
    __syncthreads();

    // ---- reverse scan, one lane per row (ppo_models.py:130-136, same op order, no fma)
    double s1 = 0.0, s2 = 0.0;
    if (tid < rows) {
        float* pv = sv + tid * a.stride;
        float* pr = sr + tid * a.stride;
        float A = 0.0f, vnext = 0.0f;
        for (int c = a.Teff - 1; c >= 0; --c) {
            const float vcur = pv[c];
            const float nv = (c < a.Teff - 1) ? vnext : 0.0f;
            const float delta = add_rn(pr[c], mul_rn(a.gamma, nv)) - vcur;
            A = add_rn(delta, mul_rn(a.gl, A));
            pr[c] = A;
            pv[c] = add_rn(A, vcur);  // returns = advantages + values
            vnext = vcur;
            s1 += double(A);
            s2 += double(A) * double(A);
        }
    }
    const double mine[TRLX_MOMENT_SLOTS] = {s1, s2, double(tid == 0 ? nel : 0), msum};
    const double rec = block_sum_multi<TRLX_MOMENT_SLOTS>(mine, red);  // (its barrier also orders
                                                                      //  the scan before write-back)

    // ---- write back advantages (raw, fp32) and returns (coalesced)
    for (int e = tid; e < nel; e += kGaeThreads) {
        const int r = e / a.Teff;
        const int c = e - r * a.Teff;
        const int64_t oi = int64_t(row0 + r) * a.Teff + c;
        a.adv[oi] = sr[r * a.stride + c];
        st_any(a.ret, a.ret_dtype, oi, sv[r * a.stride + c]);
    }
    double* my = a.partials + blockIdx.x * TRLX_MOMENT_SLOTS;
    if (!a.stats) {
        if (tid < TRLX_MOMENT_SLOTS) my[tid] = rec;
        return;
    }
    if (publish_record_last<TRLX_MOMENT_SLOTS>(my, rec, a.ticket, gridDim.x)) {
        __syncthreads();  // red[] reuse
        const double tot = reduce_records<TRLX_MOMENT_SLOTS>(a.partials, gridDim.x, red);
        if (tid < TRLX_MOMENT_SLOTS) a.stats[tid] = tot;
    }
}

static void gae_geometry(int64_t Teff, int& rpb, int& stride) {
    stride = int((Teff + 1) | 1);
    int64_t r = kGaeLdsFloats / stride;
    if (r > kGaeMaxRows) r = kGaeMaxRows;
    if (r < 1) r = 1;
    rpb = int(r);
}

// ------------------------------------------------------------------ A3 moments
constexpr int kMomThreads = 256;
constexpr int kMomPerBlock = kMomThreads * 16;

__device__ __forceinline__ double ld_moment(const void* p, int dtype, int64_t i) {
    if (dtype == 2) return double(reinterpret_cast<const int64_t*>(p)[i]);  // int64 (masks)
    return double(ld_any(p, dtype, i));
}

__global__ __launch_bounds__(kMomThreads) void k_moments_partial(const void* x, int dtype, int64_t n,
                                                                 double* partials) {
    __shared__ double red[(kMomThreads / kWave) * TRLX_MOMENT_SLOTS];
    const int64_t beg = int64_t(blockIdx.x) * kMomPerBlock;
    const int64_t end = min<int64_t>(n, beg + kMomPerBlock);
    double s1 = 0.0, s2 = 0.0;
    for (int64_t i = beg + threadIdx.x; i < end; i += kMomThreads) {
        const double v = ld_moment(x, dtype, i);
        s1 += v;
        s2 += v * v;
    }
    const double mine[TRLX_MOMENT_SLOTS] = {s1, s2, threadIdx.x == 0 ? double(end - beg) : 0.0, 0.0};
    const double rec = block_sum_multi<TRLX_MOMENT_SLOTS>(mine, red);
    if (threadIdx.x < TRLX_MOMENT_SLOTS) partials[blockIdx.x * TRLX_MOMENT_SLOTS + threadIdx.x] = rec;
}

__global__ __launch_bounds__(256) void k_moments_finalize(const double* partials, int64_t nblk,
                                                          double* stats) {
    __shared__ double red[(256 / kWave) * TRLX_MOMENT_SLOTS];
    const double tot = reduce_records<TRLX_MOMENT_SLOTS>(partials, int(nblk), red);
    if (threadIdx.x < TRLX_MOMENT_SLOTS) stats[threadIdx.x] = tot;
}

// ------------------------------------------------------------------ A4 whiten
__global__ void k_whiten_apply(const void* x, int dtype, int64_t n, const double* st, int unbiased,
                               int shift_mean, void* out, int out_dtype) {
    const double cnt = st[2];
    const double mean = st[0] / cnt;
    double m2 = st[1] - st[0] * mean;
    if (m2 < 0) m2 = 0;
    const float mu = float(mean);
    const float var = float(m2 / (unbiased ? cnt - 1.0 : cnt));
    const float rs = rsqrtf(var + 1e-8f);
    for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n;
         i += int64_t(gridDim.x) * blockDim.x) {
        float w = mul_rn(ld_any(x, dtype, i) - mu, rs);
        if (!shift_mean) w = add_rn(w, mu);
        st_any(out, out_dtype, i, w);
    }
}

static unsigned elementwise_blocks(int64_t n, int threads) {
    int64_t b = (n + threads - 1) / threads;
    if (b > 4096) b = 4096;
    if (b < 1) b = 1;
    return unsigned(b);
}

}  // namespace trlx

using namespace trlx;

extern "C" int trlx_kl_penalty_rewards(const void* lp, const void* ref_lp, int in_dtype, int64_t B,
                                       int64_t T, float beta, const float* scores,
                                       const int64_t* lengths, void* rewards, int out_dtype,
                                       void* stream) {
    TRLX_REQUIRE(lp && ref_lp && rewards, TRLX_ERR_ARG, "NULL lp/ref_lp/rewards");
    TRLX_REQUIRE(B >= 0 && T >= 0, TRLX_ERR_SHAPE, "bad shape");
    if (B * T == 0) return TRLX_OK;
    const float neg_beta = -beta;
    hipLaunchKernelGGL(k_kl_rewards, dim3(elementwise_blocks(B * T, 256)), dim3(256), 0,
                       (hipStream_t)stream, lp, ref_lp, in_dtype, B, T, neg_beta, scores, lengths,
                       rewards, out_dtype);
    return check_launch("k_kl_rewards");
}

extern "C" int64_t trlx_gae_num_blocks(int64_t B, int64_t Teff) {
    int rpb, stride;
    gae_geometry(Teff, rpb, stride);
    return (B + rpb - 1) / rpb;
}

extern "C" int trlx_gae_scan(const void* values, const void* rewards, int dtype, int64_t B,
                             int64_t T, int64_t Teff, float gamma, float lam, const float* lp,
                             const float* ref_lp, float neg_beta, const float* scores,
                             const int64_t* lengths, const int64_t* mask, float* adv_raw, void* ret,
                             int ret_dtype, void* rew_out, int rew_dtype, double* partials,
                             double* stats, unsigned* ticket, void* stream) {
    TRLX_REQUIRE(values && adv_raw && ret && partials, TRLX_ERR_ARG, "NULL values/adv/ret/partials");
    TRLX_REQUIRE(rewards || (lp && ref_lp), TRLX_ERR_ARG, "need rewards or (lp, ref_lp)");
    TRLX_REQUIRE(!stats || ticket, TRLX_ERR_ARG, "stats output needs a ticket word");
    TRLX_REQUIRE(B > 0 && Teff > 0 && Teff <= T && B * T < (1LL << 31), TRLX_ERR_SHAPE,
                 "bad shape B=%lld T=%lld Teff=%lld", (long long)B, (long long)T, (long long)Teff);
    TRLX_REQUIRE(!lp || Teff == T, TRLX_ERR_SHAPE, "fused KL reward needs response_length == T");
    GaeArgs a = {};
    a.values = values; a.rewards = rewards; a.dtype = dtype; a.B = int(B); a.T = int(T); a.Teff = int(Teff);
    a.gamma = gamma;
    a.gl = float(double(gamma) * double(lam));  // python float product, then fp32 (torch scalar)
    a.lp = lp; a.ref_lp = ref_lp; a.neg_beta = neg_beta; a.scores = scores; a.lengths = lengths;
    a.mask = mask; a.adv = adv_raw; a.ret = ret; a.ret_dtype = ret_dtype; a.rew_out = rew_out;
    a.rew_dtype = rew_dtype; a.partials = partials; a.stats = stats; a.ticket = ticket;
    gae_geometry(Teff, a.rpb, a.stride);
    const unsigned grid = unsigned((B + a.rpb - 1) / a.rpb);
    const size_t lds = size_t(2) * a.rpb * a.stride * sizeof(float);
    TRLX_REQUIRE(lds <= 64 * 1024, TRLX_ERR_SHAPE, "response length %lld too long", (long long)Teff);
    hipLaunchKernelGGL(k_gae, dim3(grid), dim3(kGaeThreads), lds, (hipStream_t)stream, a);
    return check_launch("k_gae");
}

extern "C" int64_t trlx_moments_num_blocks(int64_t n) {
    return n <= 0 ? 1 : (n + kMomPerBlock - 1) / kMomPerBlock;
}

extern "C" int trlx_moments_partial(const void* x, int dtype, int64_t n, double* partials,
                                    void* stream) {
    TRLX_REQUIRE(x && partials, TRLX_ERR_ARG, "NULL x/partials");
    TRLX_REQUIRE(dtype == TRLX_F32 || dtype == TRLX_BF16 || dtype == 2, TRLX_ERR_DTYPE, "dtype %d", dtype);
    const int64_t nb = trlx_moments_num_blocks(n);
    hipLaunchKernelGGL(k_moments_partial, dim3(unsigned(nb)), dim3(kMomThreads), 0, (hipStream_t)stream,
                       x, dtype, n, partials);
    return check_launch("k_moments_partial");
}

extern "C" int trlx_moments_finalize(const double* partials, int64_t nblk, double* stats, void* stream) {
    TRLX_REQUIRE(partials && stats && nblk > 0, TRLX_ERR_ARG, "bad partials");
    hipLaunchKernelGGL(k_moments_finalize, dim3(1), dim3(256), 0, (hipStream_t)stream, partials, nblk,
                       stats);
    return check_launch("k_moments_finalize");
}

extern "C" int trlx_whiten_apply(const void* x, int dtype, int64_t n, const double* stats, int unbiased,
                                 int shift_mean, void* out, int out_dtype, void* stream) {
    TRLX_REQUIRE(x && stats && out, TRLX_ERR_ARG, "NULL x/stats/out");
    if (n == 0) return TRLX_OK;
    hipLaunchKernelGGL(k_whiten_apply, dim3(elementwise_blocks(n, 256)), dim3(256), 0, (hipStream_t)stream,
                       x, dtype, n, stats, unbiased, shift_mean, out, out_dtype);
    return check_launch("k_whiten_apply");
}
