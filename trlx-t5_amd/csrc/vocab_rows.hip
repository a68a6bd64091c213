// Vocab-axis row kernels: fused log-softmax + gather (forward), its backward, and the
// loss-side fused forward+backward (logprob -> PPO policy gradient -> dlogits).
//
// One workgroup owns one logits row (b, t) of V elements.  The row is loaded ONCE from
// HBM into registers as 16-byte vectors (NV per thread, all loads issued up front), the
// max and sum-exp are wavefront-shuffle + LDS block reductions, and the backward /
// fused kernels write dlogits from the same registers: 1 read (+1 write) of V*s bytes per
// token, never materialising the [B,T,V] log-softmax the reference builds
// (trlx/utils/modeling.py:39).  No MFMA: there is no contraction on this path; the
// roofline is HBM bandwidth.
#include <string>

#include "ppo_math.h"

namespace trlx {

enum RowMode { kFwd = 0, kBwd = 1, kPpo = 2 };

struct RowArgs {
    const void* x0;           // logits (tensor 0)
    const void* x1;           // second logits tensor (fwd only; blockIdx.y == 1)
    int64_t B, T, V, sb, st;  // shape + token strides (elements)
    const int64_t* labels;
    int64_t lb, lt;
    // forward outputs
    void* lp0;
    void* lp1;
    int out_dtype;
    float* lse0;
    float* lse1;
    // backward inputs
    const float* lse_in;
    const void* grad;
    int grad_dtype;
    // ppo fused inputs
    const void* old_lp;
    int old_dtype;
    const float* adv;
    const double* stats;
    int unbiased;
    const int64_t* mask;
    const double* msum;
    double msum_host;
    float cliprange;
    float* lp_out;
    // gradient output (bwd / ppo)
    void* dx;
    int64_t dsb, dst;
};

template <class DT, int NV, int MODE>
__global__ __launch_bounds__(kMaxThreads) void k_vocab_rows(RowArgs a) {
    __shared__ float sh_max[kMaxThreads / kWave];
    __shared__ float sh_sum[kMaxThreads / kWave];
    typedef typename DT::elem_t E;
    constexpr int EPV = DT::kEPV;

    const int64_t row = blockIdx.x;
    const int64_t b = row / a.T, t = row - (row / a.T) * a.T;
    const int tid = threadIdx.x, nthr = blockDim.x;
    const E* xrow = reinterpret_cast<const E*>(blockIdx.y == 0 ? a.x0 : a.x1) + b * a.sb + t * a.st;
    const int64_t y = a.labels[b * a.lb + t * a.lt];
    const bool y_ok = (y >= 0) && (y < a.V);

    const RowSplit<DT> s(xrow, a.V);
    const vec4u* vp = reinterpret_cast<const vec4u*>(xrow + s.head);

    // ---- one HBM read of the row into registers (all loads in flight at once)
    vec4u v[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const int64_t i = tid + int64_t(k) * nthr;
        v[k] = (i < s.nvec) ? ld_stream(vp + i) : DT::neg_inf();
    }
    // head elements -> threads [0, head); tail elements -> the last `tail` threads
    float ex = -INFINITY;
    if (tid < s.head)
        ex = DT::load1(xrow, tid);
    else if (tid >= nthr - s.tail)
        ex = DT::load1(xrow, s.tail0 + (tid - (nthr - s.tail)));
    const float xy = y_ok ? DT::load1(xrow, y) : NAN;

    float lse, lse_l2e;
    if (MODE == kBwd) {
        lse = a.lse_in[row];
    } else {
        // ---- row max
        float m = ex;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            float f[EPV];
            DT::unpack(v[k], f);
#pragma unroll
            for (int e = 0; e < EPV; ++e) m = fmaxf(m, f[e]);
        }
        m = block_max(m, sh_max);
#pragma unroll
        for (int k = 0; k < NV; ++k) launder(v[k]);
        // ---- sum of exp(x - max)
        const float ml2e = -m * kLog2e;
        float sum = exp2_fast(fmaf(ex, kLog2e, ml2e));
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            float f[EPV];
            DT::unpack(v[k], f);
#pragma unroll
            for (int e = 0; e < EPV; ++e) sum += exp2_fast(fmaf(f[e], kLog2e, ml2e));
        }
        sum = block_sum(sum, sh_sum);
#pragma unroll
        for (int k = 0; k < NV; ++k) launder(v[k]);
        lse = m + logf(sum);
    }
    const float lp = xy - lse;

    if (MODE == kFwd) {
        if (tid == 0) {
            void* out = blockIdx.y == 0 ? a.lp0 : a.lp1;
            float* lse_out = blockIdx.y == 0 ? a.lse0 : a.lse1;
            st_any(out, a.out_dtype, row, lp);
            if (lse_out) lse_out[row] = lse;
        }
        return;
    }

    // ---- per-row gradient scale g = d loss / d lp
    float g;
    if (MODE == kBwd) {
        g = ld_any(a.grad, a.grad_dtype, row);
    } else {
        float A = a.adv[row];
        if (a.stats) {
            float mu, rstd;
            whiten_coeffs(a.stats, a.unbiased, mu, rstd);
            A = mul_rn(A - mu, rstd);
        }
        const float mval = a.mask ? float(a.mask[row]) : 1.0f;
        const double msum = a.msum ? *a.msum : a.msum_host;
        const float inv_msum = 1.0f / float(msum);  // torch: grad / mask.sum()
        const float olp = ld_any(a.old_lp, a.old_dtype, row);
        PolicyTerms pt;
        g = ppo_policy_dlp(lp, olp, A, mval, inv_msum, a.cliprange, pt);
        if (tid == 0) a.lp_out[row] = lp;
    }

    // ---- dlogits = g * (onehot(y) - exp(x - lse)), written once
    lse_l2e = -lse * kLog2e;
    E* drow = reinterpret_cast<E*>(a.dx) + b * a.dsb + t * a.dst;
    const float gy = g * (1.0f - exp2_fast(fmaf(xy, kLog2e, lse_l2e)));
    const bool same_phase = ((reinterpret_cast<uintptr_t>(drow) ^ reinterpret_cast<uintptr_t>(xrow)) & 15u) == 0;
    if (same_phase) {
        vec4u* dvp = reinterpret_cast<vec4u*>(drow + s.head);
        const int64_t iy = y_ok && y >= s.head && y < s.tail0 ? (y - s.head) / EPV : -1;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const int64_t i = tid + int64_t(k) * nthr;
            if (i < s.nvec) {
                float f[EPV];
                DT::unpack(v[k], f);
#pragma unroll
                for (int e = 0; e < EPV; ++e) f[e] = -g * exp2_fast(fmaf(f[e], kLog2e, lse_l2e));
                if (i == iy) {  // the label's vector: onehot term
                    const int ey = int(y - (s.head + i * EPV));
#pragma unroll
                    for (int e = 0; e < EPV; ++e)
                        if (e == ey) f[e] = gy;
                }
                __builtin_nontemporal_store(DT::pack(f), dvp + i);
            }
        }
    } else {
        // dlogits row not co-aligned with the logits row: element stores (correct, slower)
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const int64_t i = tid + int64_t(k) * nthr;
            if (i < s.nvec) {
                float f[EPV];
                DT::unpack(v[k], f);
#pragma unroll
                for (int e = 0; e < EPV; ++e) {
                    const int64_t j = s.head + i * EPV + e;
                    DT::store1(drow, j, j == y ? gy : -g * exp2_fast(fmaf(f[e], kLog2e, lse_l2e)));
                }
            }
        }
    }
    // head / tail elements
    int64_t jx = -1;
    if (tid < s.head)
        jx = tid;
    else if (tid >= nthr - s.tail)
        jx = s.tail0 + (tid - (nthr - s.tail));
    if (jx >= 0) DT::store1(drow, jx, jx == y ? gy : -g * exp2_fast(fmaf(ex, kLog2e, lse_l2e)));
}

// ------------------------------------------------------------------ streaming variant
// Same arithmetic, but the row is streamed through registers U vectors at a time with an
// online (max, sum-exp) instead of being held whole: small register footprint => many
// workgroups per CU keep loads continuously in flight.  Backward / fused modes make a
// second pass over the row (served from L2 / the Infinity Cache when it was just read).
__device__ __forceinline__ void online_merge(float& m, float& s, float m2, float s2) {
    const float nm = fmaxf(m, m2);
    if (nm == -INFINITY) return;  // both empty
    s = s * exp2_fast((m - nm) * kLog2e) + s2 * exp2_fast((m2 - nm) * kLog2e);
    m = nm;
}

constexpr int kStreamMaxThreads = 256;  // launch bound of the streaming kernel (register budget)

template <class DT, int U, int MODE>
__global__ __launch_bounds__(kStreamMaxThreads) void k_vocab_rows_stream(RowArgs a) {
    __shared__ float sh_m[kStreamMaxThreads / kWave];
    __shared__ float sh_s[kStreamMaxThreads / kWave];
    typedef typename DT::elem_t E;
    constexpr int EPV = DT::kEPV;
    const int64_t row = blockIdx.x;
    const int64_t b = row / a.T, t = row - (row / a.T) * a.T;
    const int tid = threadIdx.x, nthr = blockDim.x;
    const E* xrow = reinterpret_cast<const E*>(blockIdx.y == 0 ? a.x0 : a.x1) + b * a.sb + t * a.st;
    const int64_t y = a.labels[b * a.lb + t * a.lt];
    const bool y_ok = (y >= 0) && (y < a.V);
    const RowSplit<DT> s(xrow, a.V);
    const vec4u* vp = reinterpret_cast<const vec4u*>(xrow + s.head);
    float ex = -INFINITY;
    if (tid < s.head)
        ex = DT::load1(xrow, tid);
    else if (tid >= nthr - s.tail)
        ex = DT::load1(xrow, s.tail0 + (tid - (nthr - s.tail)));
    const float xy = y_ok ? DT::load1(xrow, y) : NAN;

    float lse;
    if (MODE == kBwd) {
        lse = a.lse_in[row];
    } else {
        float m = ex, sum = (ex == -INFINITY) ? 0.0f : 1.0f;
        for (int64_t base = tid; base < s.nvec; base += int64_t(nthr) * U) {
            vec4u v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t i = base + int64_t(u) * nthr;
                v[u] = (i < s.nvec) ? ld_stream(vp + i) : DT::neg_inf();
            }
            float mx = -INFINITY;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                float f[EPV];
                DT::unpack(v[u], f);
#pragma unroll
                for (int e = 0; e < EPV; ++e) mx = fmaxf(mx, f[e]);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) launder(v[u]);
            const float nm = fmaxf(m, mx);
            if (nm == -INFINITY) continue;
            sum *= exp2_fast((m - nm) * kLog2e);
            const float nml2e = -nm * kLog2e;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                float f[EPV];
                DT::unpack(v[u], f);
#pragma unroll
                for (int e = 0; e < EPV; ++e) sum += exp2_fast(fmaf(f[e], kLog2e, nml2e));
            }
            m = nm;
        }
        // wave combine, then fixed-order cross-wave combine
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const float m2 = __shfl_xor(m, off, kWave), s2 = __shfl_xor(sum, off, kWave);
            online_merge(m, sum, m2, s2);
        }
        if ((tid & (kWave - 1)) == 0) {
            sh_m[tid / kWave] = m;
            sh_s[tid / kWave] = sum;
        }
        __syncthreads();
        m = sh_m[0];
        sum = sh_s[0];
        for (int w = 1; w < nthr / kWave; ++w) online_merge(m, sum, sh_m[w], sh_s[w]);
        lse = m + logf(sum);
    }
    const float lp = xy - lse;
    if (MODE == kFwd) {
        if (tid == 0) {
            void* out = blockIdx.y == 0 ? a.lp0 : a.lp1;
            float* lse_out = blockIdx.y == 0 ? a.lse0 : a.lse1;
            st_any(out, a.out_dtype, row, lp);
            if (lse_out) lse_out[row] = lse;
        }
        return;
    }
    float g;
    if (MODE == kBwd) {
        g = ld_any(a.grad, a.grad_dtype, row);
    } else {
        float A = a.adv[row];
        if (a.stats) {
            float mu, rstd;
            whiten_coeffs(a.stats, a.unbiased, mu, rstd);
            A = mul_rn(A - mu, rstd);
        }
        const float mval = a.mask ? float(a.mask[row]) : 1.0f;
        const double msum = a.msum ? *a.msum : a.msum_host;
        const float inv_msum = 1.0f / float(msum);
        const float olp = ld_any(a.old_lp, a.old_dtype, row);
        PolicyTerms pt;
        g = ppo_policy_dlp(lp, olp, A, mval, inv_msum, a.cliprange, pt);
        if (tid == 0) a.lp_out[row] = lp;
    }
    const float lse_l2e = -lse * kLog2e;
    E* drow = reinterpret_cast<E*>(a.dx) + b * a.dsb + t * a.dst;
    const float gy = g * (1.0f - exp2_fast(fmaf(xy, kLog2e, lse_l2e)));
    const bool same_phase = ((reinterpret_cast<uintptr_t>(drow) ^ reinterpret_cast<uintptr_t>(xrow)) & 15u) == 0;
    const int64_t iy = y_ok && y >= s.head && y < s.tail0 ? (y - s.head) / EPV : -1;
    vec4u* dvp = reinterpret_cast<vec4u*>(drow + s.head);
    for (int64_t base = tid; base < s.nvec; base += int64_t(nthr) * U) {
        vec4u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = base + int64_t(u) * nthr;
            if (i < s.nvec) v[u] = vp[i];  // second touch: cached read
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = base + int64_t(u) * nthr;
            if (i >= s.nvec) continue;
            float f[EPV];
            DT::unpack(v[u], f);
#pragma unroll
            for (int e = 0; e < EPV; ++e) f[e] = -g * exp2_fast(fmaf(f[e], kLog2e, lse_l2e));
            if (same_phase) {
                if (i == iy) {
                    const int ey = int(y - (s.head + i * EPV));
#pragma unroll
                    for (int e = 0; e < EPV; ++e)
                        if (e == ey) f[e] = gy;
                }
                __builtin_nontemporal_store(DT::pack(f), dvp + i);
            } else {
#pragma unroll
                for (int e = 0; e < EPV; ++e) {
                    const int64_t j = s.head + i * EPV + e;
                    DT::store1(drow, j, j == y ? gy : f[e]);
                }
            }
        }
    }
    int64_t jx = -1;
    if (tid < s.head)
        jx = tid;
    else if (tid >= nthr - s.tail)
        jx = s.tail0 + (tid - (nthr - s.tail));
    if (jx >= 0) DT::store1(drow, jx, jx == y ? gy : -g * exp2_fast(fmaf(ex, kLog2e, lse_l2e)));
}

// ------------------------------------------------------------------ launch geometry
// Vectors per thread (NV) are compile-time so the row lives in registers; threads per
// block = the smallest multiple of 64 that covers the row with NV vectors.
struct Geometry {
    int nv;
    int threads;
};
static int g_resident_threads = 0;  // preferred workgroup size for resident rows (0 = auto)

// Register-resident geometry: NV (compile-time vectors per thread, from kNVs) and the
// workgroup size.  Default: 512-thread workgroups (8 waves) -- measured on MI355X (C2,
// bf16 V=50257) to keep 3 rows in flight per CU at ~71 VGPRs, 6.7 TB/s for the forward;
// rows too long for 16 vectors x 512 threads use 1024 threads, then the streaming kernel.
static const int kNVs[] = {1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 13, 16};

static Geometry pick_geometry(int64_t V, int elem_bytes, bool allow_1024) {
    const int epv = 16 / elem_bytes;
    const int64_t nvec = V / epv + 1;  // upper bound incl. head/tail peeling
    const int prefs[2] = {g_resident_threads > 0 ? g_resident_threads : 512, kMaxThreads};
    for (int pi = 0; pi < (allow_1024 ? 2 : 1); ++pi) {
        const int pref = prefs[pi];
        const int64_t need = (nvec + pref - 1) / pref;
        for (int nv : kNVs) {
            if (nv < need) continue;
            int64_t thr = (nvec + nv - 1) / nv;
            thr = ((thr + kWave - 1) / kWave) * kWave;
            return {nv, int(thr < kWave ? kWave : thr)};
        }
        if (g_resident_threads > 0) break;  // a fixed size that does not fit -> streaming
    }
    return {0, 0};
}

// Tuning knobs (trlx_set_tuning): 0 = automatic.
static int g_row_variant = 0;   // 1 = register-resident rows, 2 = streaming rows
static int g_stream_threads = 0;
static int g_stream_unroll = 0;

template <int MODE, class DT>
static int launch_rows_dt(const RowArgs& a, int nten, hipStream_t stream) {
    const dim3 grid(unsigned(a.B * a.T), unsigned(nten));
    // Forward (read-only): resident rows while a 512-thread workgroup holds the row, else
    // streaming (measured: 1024-thread resident rows lose ~20% to streaming on fp32 V=50257).
    // Backward / fused (read + write): resident up to 1024 threads (one read instead of two).
    const Geometry g = pick_geometry(a.V, sizeof(typename DT::elem_t), MODE != kFwd || g_resident_threads > 0);
    const int variant = g_row_variant ? g_row_variant : (g.nv > 0 ? 1 : 2);
    if (variant == 2 || g.nv == 0) {
        const int thr = g_stream_threads ? g_stream_threads : kStreamMaxThreads;
        const int unroll = g_stream_unroll ? g_stream_unroll : 4;
        if (unroll == 8)
            hipLaunchKernelGGL((k_vocab_rows_stream<DT, 8, MODE>), grid, dim3(thr), 0, stream, a);
        else if (unroll == 2)
            hipLaunchKernelGGL((k_vocab_rows_stream<DT, 2, MODE>), grid, dim3(thr), 0, stream, a);
        else
            hipLaunchKernelGGL((k_vocab_rows_stream<DT, 4, MODE>), grid, dim3(thr), 0, stream, a);
        return check_launch("k_vocab_rows_stream");
    }
    const dim3 block(g.threads);
#define TRLX_RESIDENT_CASE(N) \
    case N: hipLaunchKernelGGL((k_vocab_rows<DT, N, MODE>), grid, block, 0, stream, a); break;
    switch (g.nv) {
        TRLX_RESIDENT_CASE(1) TRLX_RESIDENT_CASE(2) TRLX_RESIDENT_CASE(3) TRLX_RESIDENT_CASE(4)
        TRLX_RESIDENT_CASE(5) TRLX_RESIDENT_CASE(6) TRLX_RESIDENT_CASE(7) TRLX_RESIDENT_CASE(8)
        TRLX_RESIDENT_CASE(10) TRLX_RESIDENT_CASE(12) TRLX_RESIDENT_CASE(13) TRLX_RESIDENT_CASE(16)
        default: TRLX_REQUIRE(false, TRLX_ERR_SHAPE, "no resident geometry for NV=%d", g.nv);
    }
#undef TRLX_RESIDENT_CASE
    return check_launch("k_vocab_rows");
}

template <int MODE>
static int launch_rows(const RowArgs& a, int dtype, int nten, hipStream_t stream) {
    if (a.B * a.T == 0) return TRLX_OK;
    if (dtype == TRLX_BF16) return launch_rows_dt<MODE, BF16T>(a, nten, stream);
    return launch_rows_dt<MODE, F32T>(a, nten, stream);
}

static int check_rows(const RowArgs& a, int dtype) {
    TRLX_REQUIRE(dtype == TRLX_F32 || dtype == TRLX_BF16, TRLX_ERR_DTYPE, "logits dtype %d unsupported", dtype);
    TRLX_REQUIRE(a.B >= 0 && a.T >= 0 && a.V > 0, TRLX_ERR_SHAPE, "bad shape B=%lld T=%lld V=%lld",
                 (long long)a.B, (long long)a.T, (long long)a.V);
    TRLX_REQUIRE(a.B * a.T <= 0x7fffffffLL, TRLX_ERR_SHAPE, "too many rows");
    TRLX_REQUIRE(a.x0 && a.labels, TRLX_ERR_ARG, "NULL logits/labels");
    return TRLX_OK;
}

}  // namespace trlx

using namespace trlx;

extern "C" int trlx_lsm_gather_fwd(const void* x0, const void* x1, int dtype, int64_t B, int64_t T,
                                   int64_t V, int64_t sb, int64_t st, const int64_t* labels,
                                   int64_t lb, int64_t lt, void* out_lp0, void* out_lp1,
                                   int out_dtype, float* out_lse0, float* out_lse1, void* stream) {
    RowArgs a = {};
    a.x0 = x0; a.x1 = x1; a.B = B; a.T = T; a.V = V; a.sb = sb; a.st = st;
    a.labels = labels; a.lb = lb; a.lt = lt;
    a.lp0 = out_lp0; a.lp1 = out_lp1; a.out_dtype = out_dtype; a.lse0 = out_lse0; a.lse1 = out_lse1;
    if (B * T == 0 && B >= 0 && T >= 0) return TRLX_OK;  // empty batch: nothing to launch
    int rc = check_rows(a, dtype);
    if (rc) return rc;
    TRLX_REQUIRE(out_lp0 && (!x1 || out_lp1), TRLX_ERR_ARG, "NULL logprob output");
    TRLX_REQUIRE(out_dtype == TRLX_F32 || out_dtype == TRLX_BF16, TRLX_ERR_DTYPE, "out dtype");
    return launch_rows<kFwd>(a, dtype, x1 ? 2 : 1, (hipStream_t)stream);
}

extern "C" int trlx_lsm_gather_bwd(const void* x, int dtype, int64_t B, int64_t T, int64_t V,
                                   int64_t sb, int64_t st, const int64_t* labels, int64_t lb,
                                   int64_t lt, const float* lse, const void* grad, int grad_dtype,
                                   void* dx, int64_t dsb, int64_t dst, void* stream) {
    RowArgs a = {};
    a.x0 = x; a.B = B; a.T = T; a.V = V; a.sb = sb; a.st = st; a.labels = labels; a.lb = lb; a.lt = lt;
    a.lse_in = lse; a.grad = grad; a.grad_dtype = grad_dtype; a.dx = dx; a.dsb = dsb; a.dst = dst;
    if (B * T == 0 && B >= 0 && T >= 0) return TRLX_OK;  // empty batch: nothing to launch
    int rc = check_rows(a, dtype);
    if (rc) return rc;
    TRLX_REQUIRE(lse && grad && dx, TRLX_ERR_ARG, "NULL lse/grad/dx");
    return launch_rows<kBwd>(a, dtype, 1, (hipStream_t)stream);
}

extern "C" int trlx_ppo_policy_fused(const void* x, int dtype, int64_t B, int64_t T, int64_t V,
                                     int64_t sb, int64_t st, const int64_t* labels, int64_t lb,
                                     int64_t lt, const void* old_lp, int old_dtype, const float* adv,
                                     const double* stats, int unbiased, const int64_t* mask,
                                     const double* msum, double msum_host, float cliprange,
                                     float* lp_out, void* dx, int64_t dsb, int64_t dst, void* stream) {
    RowArgs a = {};
    a.x0 = x; a.B = B; a.T = T; a.V = V; a.sb = sb; a.st = st; a.labels = labels; a.lb = lb; a.lt = lt;
    a.old_lp = old_lp; a.old_dtype = old_dtype; a.adv = adv; a.stats = stats; a.unbiased = unbiased;
    a.mask = mask; a.msum = msum; a.msum_host = msum_host; a.cliprange = cliprange;
    a.lp_out = lp_out; a.dx = dx; a.dsb = dsb; a.dst = dst;
    if (B * T == 0 && B >= 0 && T >= 0) return TRLX_OK;  // empty batch: nothing to launch
    int rc = check_rows(a, dtype);
    if (rc) return rc;
    TRLX_REQUIRE(old_lp && adv && lp_out && dx, TRLX_ERR_ARG, "NULL old_lp/adv/lp_out/dx");
    TRLX_REQUIRE(msum || msum_host > 0, TRLX_ERR_ARG, "mask sum must be positive");
    return launch_rows<kPpo>(a, dtype, 1, (hipStream_t)stream);
}

extern "C" int trlx_set_tuning(const char* key, int64_t value) {
    const std::string k = key ? key : "";
    if (k == "row_variant") g_row_variant = int(value);
    else if (k == "resident_threads") {
        TRLX_REQUIRE(value == 0 || (value % kWave == 0 && value <= kMaxThreads), TRLX_ERR_ARG,
                     "resident_threads must be a multiple of 64 <= %d", kMaxThreads);
        g_resident_threads = int(value);
    }
    else if (k == "stream_threads") {
        TRLX_REQUIRE(value == 0 || (value % kWave == 0 && value <= kStreamMaxThreads), TRLX_ERR_ARG,
                     "stream_threads must be a multiple of 64 <= %d", kStreamMaxThreads);
        g_stream_threads = int(value);
    } else if (k == "stream_unroll") {
        TRLX_REQUIRE(value == 0 || value == 2 || value == 4 || value == 8, TRLX_ERR_ARG, "stream_unroll: 2, 4 or 8");
        g_stream_unroll = int(value);
    }
    else {
        set_error("unknown tuning key '%s'", k.c_str());
        return TRLX_ERR_ARG;
    }
    return TRLX_OK;
}
