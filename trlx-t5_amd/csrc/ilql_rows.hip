// ILQL loss (A10): ILQLConfig.loss of trlx/model/nn/ilql_models.py:52-116 with its autograd,
// as three launches over the batch (C ABI: trlx_ilql_* in include/trlx_t5_amd.h).
//
//   k_ilql_prep      n_nonterminal = max(1, Σ dones[:, :-1]) (:67-68) and
//                    Σ attention_mask[:, 1:] (:104) -> workspace (fp64); a few blocks, the
//                    last to arrive reducing their records in fixed order
//   k_ilql_rows      one workgroup per vocab row — the logits rows (AWAC cross-entropy,
//                    :98-105) and the Q-head rows (CQL cross-entropy :87-96 + TD loss
//                    :63-74); the row is read ONCE into VGPRs (16-B buffer loads, all in
//                    flight), max / Σexp are wave-shuffle + LDS reductions, and the row's
//                    gradient g·(onehot − softmax) (+ the TD gradient at the action) is
//                    written from the same registers.  Thread 0 gathers the target-Q heads
//                    at the action for the expectile V loss (:76-83) and writes d loss/d vs.
//   k_ilql_finalize  fixed-order fp64 sums of the per-row records -> the five losses of
//                    the reference's stats dict (:109-113); blocks over contiguous row
//                    ranges, the last to arrive reducing their records in fixed order.
// (Both were single-workgroup launches: 10 + 20 us of one CU's bandwidth per C5 step.)
// HBM: one read + one write of every logits / Q row (2·V·s bytes per row); target-Q rows
// cost two scalar gathers.  No MFMA: nothing here is a contraction.
#include <algorithm>

#include "common.h"

namespace trlx {

constexpr int kIlqlRec = 4;  // floats per row record: {ce·weight, td², v-loss, 0}
constexpr int kIlqlRedThreads = 256;     // prep / finalize workgroups
constexpr int kIlqlRedMaxBlocks = 128;
constexpr int kIlqlPrepPerBlock = 256;   // dones / attention elements per prep block (C5: 10.8 -> 5.4 us vs 2048)
constexpr int kIlqlFinPerBlock = 1024;   // row records per finalize block (256 / 512: 17 / 14 us vs 12)

// workspace: double[2] {n_nonterminal, Σ attention[:, 1:]} | float[R][kIlqlRec] | (16-B
// aligned) uint32 tickets[4] | double prep_rec[128][2] | double fin_rec[128][6].  The tickets
// must be zero before the first launch (the workspace is zero-filled once; the last block of
// each reduction re-arms its ticket).
__host__ __device__ inline int64_t ilql_num_rows(int64_t B, int64_t L, int64_t A, int nq) {
    return B * L + int64_t(nq) * B * A;
}
__device__ __forceinline__ const double* ilql_sums(const trlx_ilql_args& a) {
    return static_cast<const double*>(a.workspace);
}
__device__ __forceinline__ float* ilql_recs(const trlx_ilql_args& a) {
    return reinterpret_cast<float*>(static_cast<char*>(a.workspace) + 16);
}
__host__ __device__ inline int64_t ilql_red_offset(int64_t R) {  // tickets, then the block records
    return (16 + int64_t(sizeof(float)) * kIlqlRec * R + 15) & ~int64_t(15);
}
__host__ __device__ inline int ilql_red_blocks(int64_t n, int per) {
    const int64_t b = (n + per - 1) / per;
    return int(b < 1 ? 1 : (b > kIlqlRedMaxBlocks ? kIlqlRedMaxBlocks : b));
}
struct IlqlRed {
    unsigned* tickets;
    double* prep_rec;  // [kIlqlRedMaxBlocks][2]
    double* fin_rec;   // [kIlqlRedMaxBlocks][6]
};
__device__ __forceinline__ IlqlRed ilql_red(const trlx_ilql_args& a) {
    char* base = static_cast<char*>(a.workspace) + ilql_red_offset(ilql_num_rows(a.B, a.L, a.A, a.nq));
    IlqlRed r;
    r.tickets = reinterpret_cast<unsigned*>(base);
    r.prep_rec = reinterpret_cast<double*>(base + 16);
    r.fin_rec = reinterpret_cast<double*>(base + 16 + kIlqlRedMaxBlocks * 2 * sizeof(double));
    return r;
}

// Row r of the launch: [0, B·L) logits rows (b, t); then nq blocks of B·A Q-head rows (b, a).
struct IlqlRowId {
    int head;       // -1: logits row; i: Q head i
    int64_t b, t;   // t = token index (logits) or action index (Q heads)
};
__device__ __forceinline__ IlqlRowId ilql_decode(const trlx_ilql_args& a, int64_t r) {
    IlqlRowId o;
    const int64_t nl = a.B * a.L;
    if (r < nl) {
        o.head = -1;
        o.b = r / a.L;
        o.t = r - o.b * a.L;
    } else {
        r -= nl;
        const int64_t na = a.B * a.A;
        o.head = int(r / na);
        r -= int64_t(o.head) * na;
        o.b = r / a.A;
        o.t = r - o.b * a.A;
    }
    return o;
}

// ------------------------------------------------------------------ prep
// Block b sums elements [b·chunk, (b+1)·chunk) of dones[:, :-1] and of attention[:, 1:] (same
// chunk bounds for both index spaces), one fp64 record per block; the last block to arrive
// reduces the records in block order.
__global__ __launch_bounds__(kIlqlRedThreads) void k_ilql_prep(trlx_ilql_args a) {
    __shared__ double sh[(kIlqlRedThreads / kWave) * 2];
    const int64_t S = a.A + 1, L1 = a.L - 1;
    const int64_t nd = a.B * a.A, na = a.B * L1;
    const int64_t chunk = (max(nd, na) + gridDim.x - 1) / gridDim.x;
    const int64_t i0 = int64_t(blockIdx.x) * chunk, i1 = i0 + chunk;
    double st = 0.0, sa = 0.0;
    for (int64_t i = i0 + threadIdx.x; i < min(i1, nd); i += blockDim.x) {
        const int64_t b = i / a.A;
        st += double(a.dones[b * S + (i - b * a.A)]);
    }
    for (int64_t i = i0 + threadIdx.x; i < min(i1, na); i += blockDim.x) {
        const int64_t b = i / L1;
        sa += double(a.attention_mask[b * a.L + 1 + (i - b * L1)]);
    }
    const double v[2] = {st, sa};
    const double r = block_sum_multi<2>(v, sh);
    const IlqlRed red = ilql_red(a);
    if (publish_record_last<2>(red.prep_rec + blockIdx.x * 2, r, red.tickets + 0, gridDim.x)) {
        __syncthreads();  // sh[] reuse
        const double t = reduce_records<2>(red.prep_rec, int(gridDim.x), sh);
        double* out = static_cast<double*>(a.workspace);
        if (threadIdx.x == 0) out[0] = t > 1.0 ? t : 1.0;  // max(1, terminal_mask.sum())
        if (threadIdx.x == 1) out[1] = t;
    }
}

// ------------------------------------------------------------------ rows
// Per-row scalars (wave-uniform), parked in LDS by thread 0 while the row loads fly.
struct IlqlRowScalars {
    float g;    // d loss / d log_softmax[y] of the row's cross-entropy term (= -weight·scale)
    float w;    // the CE weight (attention / terminal mask)
    float Qt;   // TD target r + γ·V_next·done (Q rows)
    float inv_n;
};

// NL > 0: split residency for long fp32 rows, as k_vocab_rows (vocab_rows.hip): the last NL
// vector steps live in LDS (DMA), 512 threads, two rows in flight per CU.
template <class DT, int NV, int NL = 0>
__global__ __launch_bounds__(NL ? 512 : kMaxThreads, NL ? 4 : 1) void k_ilql_rows(trlx_ilql_args a) {
    __shared__ float sh_max[kMaxThreads / kWave];
    __shared__ float sh_sum[kMaxThreads / kWave];
    __shared__ float s_sc[4];
    typedef typename DT::elem_t E;
    constexpr int EPV = DT::kEPV;
    const int tid = threadIdx.x, nthr = blockDim.x;
    const IlqlRowId id = ilql_decode(a, blockIdx.x);
    const int64_t S = a.A + 1;
    float* rec = ilql_recs(a) + int64_t(blockIdx.x) * kIlqlRec;

    const E* x;
    E* dx;
    int64_t y;
    // Rows whose every loss term carries a zero weight have a zero gradient and add nothing to
    // the sums: the last logits position (logits[:, :-1] only), a logits row whose next token
    // is padding (AWAC weight attention_mask[b, t+1] = 0, ilql_models.py:98-105) and a Q row of
    // a terminal action (CQL and TD weights dones[b, a] = 0, :63-74 and :87-96; the V loss of
    // head 0 too, :76-83).  Such a row is written as zeros without being read (a masked row of
    // non-finite logits made the reference's loss NaN through NaN·0).  The
    // per-row mask load runs only when prep found a zero weight (its sums short of the counts).
    bool skip = id.head < 0 && id.t == a.L - 1;
    if (!skip) {
        const double* sums = ilql_sums(a);
        const bool masked = sums[0] != double(a.B * a.A) || sums[1] != double(a.B * (a.L - 1));
        if (masked)
            skip = id.head < 0 ? a.attention_mask[id.b * a.L + id.t + 1] == 0 : a.dones[id.b * S + id.t] == 0;
    }
    if (id.head < 0) {
        x = static_cast<const E*>(a.logits) + id.b * a.logits_sb + id.t * a.logits_st;
        dx = static_cast<E*>(a.dlogits) + id.b * a.dlogits_sb + id.t * a.dlogits_st;
    } else {
        dx = static_cast<E*>(a.dq[id.head]) + id.b * a.dq_sb[id.head] + id.t * a.dq_st[id.head];
    }
    if (skip) {
        const RowSplit<DT> s(dx, a.V);
        const __amdgpu_buffer_rsrc_t rout = make_rsrc(dx + s.head, uint32_t(s.nvec) * 16u);
        const vec4u z = vec4u_make(0u, 0u, 0u, 0u);
        for (int i = tid; i < int(s.nvec); i += nthr)
            __builtin_amdgcn_raw_buffer_store_b128(z, rout, i * 16, 0, kAuxNT);
        if (tid < s.head) DT::store1(dx, tid, 0.0f);
        if (tid < s.tail) DT::store1(dx, s.tail0 + tid, 0.0f);
        if (tid < kIlqlRec) rec[tid] = 0.0f;
        if (id.head == 0 && tid == 0) {  // d loss_v / d vs of state (b, t): weight dones[b, t] = 0
            a.dvs[id.b * S + id.t] = 0.0f;
            if (id.t == a.A - 1) a.dvs[id.b * S + a.A] = 0.0f;  // V_next is detached
        }
        return;
    }
    if (id.head < 0) {
        y = a.input_ids[id.b * a.L + id.t + 1];
    } else {
        const int h = id.head;
        x = static_cast<const E*>(a.q[h]) + id.b * a.q_sb[h] + id.t * a.q_st[h];
        const int64_t ix = a.actions_ixs[id.b * a.A + id.t];
        y = (ix >= 0 && ix < a.L - 1) ? a.input_ids[id.b * a.L + 1 + ix] : -1;  // no OOB gather
    }
    const bool y_ok = y >= 0 && y < a.V;
    if (tid == 0) {  // row-independent scalars while the row loads are in flight
        const double* sums = ilql_sums(a);
        IlqlRowScalars p;
        if (id.head < 0) {
            p.w = float(a.attention_mask[id.b * a.L + id.t + 1]);
            p.g = -mul_rn(a.awac_scale / float(sums[1]), p.w);  // awac·1 / Σattn, ·attn
            p.Qt = 0.0f;
            p.inv_n = 0.0f;
        } else {
            const float nf = float(sums[0]);
            p.w = float(a.dones[id.b * S + id.t]);
            p.g = -mul_rn(a.cql_scale / nf, p.w);
            const float vn = mul_rn(ld_any(a.vs, a.vs_dtype, id.b * S + id.t + 1),
                                    float(a.dones[id.b * S + id.t + 1]));
            p.Qt = add_rn(ld_any(a.rewards, a.rewards_dtype, id.b * a.A + id.t), mul_rn(a.gamma, vn));
            p.inv_n = 1.0f / nf;
        }
        s_sc[0] = p.g; s_sc[1] = p.w; s_sc[2] = p.Qt; s_sc[3] = p.inv_n;
    }

    const RowSplit<DT> s(x, a.V);
    const int nvec = int(s.nvec);
    const __amdgpu_buffer_rsrc_t rin = make_rsrc(x + s.head, uint32_t(nvec) * 16u);
    const int shift = line_shift(x + s.head);  // whole 256-B spans per wave instruction (common.h)
    const int voff = (tid - shift) * 16;       // step-major vector order (vocab_rows.hip)
    vec4u v[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k)
        v[k] = __builtin_amdgcn_raw_buffer_load_b128(rin, launder_int(voff) + k * nthr * 16, 0, kAuxNT);
    __shared__ __attribute__((aligned(16))) vec4u lds_row[NL > 0 ? NL * 512 : 1];
    if constexpr (NL > 0) {  // vector steps NV .. NV+NL-1 -> lds_row[kk][tid]
        const char* body = reinterpret_cast<const char*>(x + s.head);
        char* lbase = reinterpret_cast<char*>(lds_row) + (tid >> 6) * 1024;
#pragma unroll
        for (int kk = 0; kk < NL; ++kk) {
            const int i = tid - shift + (NV + kk) * nthr;
            const int ic = unsigned(i) < unsigned(nvec) ? i : 0;
            __builtin_amdgcn_global_load_lds(body + int64_t(ic) * 16,
                                             (__attribute__((address_space(3))) void*)(lbase + kk * 8192), 16, 0, 0);
        }
    }
    const float xy = y_ok ? DT::load1(x, y) : NAN;
    int64_t je = -1;  // head element -> threads [0, head); tail element -> the last `tail` threads
    if (tid < s.head) je = tid;
    else if (tid >= nthr - s.tail) je = s.tail0 + (tid - (nthr - s.tail));
    const float ex = je >= 0 ? DT::load1(x, je) : -INFINITY;

    float m = ex;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        float f[EPV];
        DT::unpack(v[k], f);
        float mk = f[0];
#pragma unroll
        for (int e = 1; e < EPV; ++e) mk = fmaxf(mk, f[e]);
        m = (unsigned(tid - shift + k * nthr) < unsigned(nvec)) ? fmaxf(m, mk) : m;
    }
    if constexpr (NL > 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this lane's DMAs (it reads only its own)
#pragma unroll
        for (int kk = 0; kk < NL; ++kk) {
            float f[EPV];
            DT::unpack(lds_row[kk * 512 + tid], f);
            float mk = f[0];
#pragma unroll
            for (int e = 1; e < EPV; ++e) mk = fmaxf(mk, f[e]);
            m = (unsigned(tid - shift + (NV + kk) * nthr) < unsigned(nvec)) ? fmaxf(m, mk) : m;
        }
    }
    m = block_max(m, sh_max);
#pragma unroll
    for (int k = 0; k < NV; ++k) launder(v[k]);
    const float ml2e = -m * kLog2e;
    const f32x2 l2e2 = f2_splat(kLog2e), ml2e2 = f2_splat(ml2e), zero2 = f2_splat(0.0f);
    f32x2 acc = {exp2_fast(fmaf(ex, kLog2e, ml2e)), 0.0f};  // packed pairs, as the vocab rows
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        float f[EPV];
        DT::unpack(v[k], f);
        const f32x2 sk = exp_pair_sum(f, l2e2, ml2e2);
        acc += (unsigned(tid - shift + k * nthr) < unsigned(nvec)) ? sk : zero2;
    }
    if constexpr (NL > 0) {
#pragma unroll
        for (int kk = 0; kk < NL; ++kk) {
            float f[EPV];
            DT::unpack(lds_row[kk * 512 + tid], f);
            const f32x2 sk = exp_pair_sum(f, l2e2, ml2e2);
            acc += (unsigned(tid - shift + (NV + kk) * nthr) < unsigned(nvec)) ? sk : zero2;
        }
    }
    float sum = acc.x + acc.y;
    sum = block_sum(sum, sh_sum);
#pragma unroll
    for (int k = 0; k < NV; ++k) launder(v[k]);
    const float lse = m + logf(sum);

    // (the reductions' barriers order thread 0's s_sc writes before these reads)
    const float g = s_sc[0];
    float dQ = 0.0f, d = 0.0f;
    if (id.head >= 0) {  // TD term: ((Q - Qt)·w)², its gradient lands on the action element
        const float w = s_sc[1];
        d = mul_rn(xy - s_sc[2], w);
        dQ = mul_rn(mul_rn(s_sc[3], mul_rn(2.0f, d)), w);
    }
    const float lse_l2e = -lse * kLog2e;
    const float gy = add_rn(g * (1.0f - exp2_fast(fmaf(xy, kLog2e, lse_l2e))), dQ);
    if (je >= 0) DT::store1(dx, je, je == y ? gy : -g * exp2_fast(fmaf(ex, kLog2e, lse_l2e)));
    const __amdgpu_buffer_rsrc_t rout = make_rsrc(dx + s.head, uint32_t(nvec) * 16u);
    const int iy = y_ok && y >= s.head && y < s.tail0 ? int((y - s.head) / EPV) : -1;
    const f32x2 c2 = f2_splat(lse_l2e), ng2 = f2_splat(-g);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const int i = tid - shift + k * nthr;  // lanes outside the body: range-checked away
        float f[EPV];
        DT::unpack(v[k], f);
        neg_g_exp_pairs(f, l2e2, c2, ng2);
        if (i == iy) {
            const int ey = int(y - (s.head + int64_t(i) * EPV));
#pragma unroll
            for (int e = 0; e < EPV; ++e)
                if (e == ey) f[e] = gy;
        }
        __builtin_amdgcn_raw_buffer_store_b128(DT::pack(f), rout, launder_int(voff) + k * nthr * 16, 0, kAuxNT);
    }
    if constexpr (NL > 0) {
#pragma unroll
        for (int kk = 0; kk < NL; ++kk) {
            const int i = tid - shift + (NV + kk) * nthr;
            float f[EPV];
            DT::unpack(lds_row[kk * 512 + tid], f);
            neg_g_exp_pairs(f, l2e2, c2, ng2);
            if (i == iy) {
                const int ey = int(y - (s.head + int64_t(i) * EPV));
#pragma unroll
                for (int e = 0; e < EPV; ++e)
                    if (e == ey) f[e] = gy;
            }
            __builtin_amdgcn_raw_buffer_store_b128(DT::pack(f), rout, launder_int(voff) + (NV + kk) * nthr * 16, 0,
                                                   kAuxNT);
        }
    }

    if (tid == 0) {
        const float w = s_sc[1];
        const float ce = lse - xy;  // cross_entropy = -log_softmax[y]
        float vl = 0.0f;
        if (id.head == 0) {  // expectile V loss + d loss / d vs for state (b, t)
            const int64_t* ai = a.actions_ixs;
            (void)ai;
            float tQ = y_ok ? DT::load1(static_cast<const E*>(a.tq[0]) + id.b * a.tq_sb[0] + id.t * a.tq_st[0], y)
                            : NAN;
            if (a.nq > 1) {
                const float t1 = y_ok ? DT::load1(static_cast<const E*>(a.tq[1]) + id.b * a.tq_sb[1] +
                                                      id.t * a.tq_st[1], y)
                                      : NAN;
                tQ = (tQ != tQ || t1 != t1) ? NAN : fminf(tQ, t1);  // torch.minimum propagates NaN
            }
            const float V = ld_any(a.vs, a.vs_dtype, id.b * S + id.t);
            const float diff = tQ - V;
            const float sq = mul_rn(diff, diff);
            const float w1 = tQ >= V ? a.tau : 0.0f;
            const float w2 = tQ < V ? float(1.0 - double(a.tau)) : 0.0f;
            vl = mul_rn(add_rn(mul_rn(w1, sq), mul_rn(w2, sq)), w);
            const float gw = mul_rn(s_sc[3], w);
            const float two_diff = mul_rn(2.0f, diff);
            a.dvs[id.b * S + id.t] = add_rn(-mul_rn(mul_rn(gw, w1), two_diff), -mul_rn(mul_rn(gw, w2), two_diff));
            if (id.t == a.A - 1) a.dvs[id.b * S + a.A] = 0.0f;  // V_next is detached
        }
        rec[0] = mul_rn(ce, w);
        rec[1] = mul_rn(d, d);
        rec[2] = vl;
        rec[3] = 0.0f;
    }
}

// ------------------------------------------------------------------ finalize
// Block b sums the row records [b·chunk, (b+1)·chunk); the last block to arrive reduces the
// block records in block order and emits the losses.
__global__ __launch_bounds__(kIlqlRedThreads) void k_ilql_finalize(trlx_ilql_args a) {
    __shared__ double sh[(kIlqlRedThreads / kWave) * 6];
    __shared__ double tot[6];
    const int64_t nl = a.B * a.L, na = a.B * a.A;
    const int64_t R = ilql_num_rows(a.B, a.L, a.A, a.nq);
    const int64_t chunk = (R + gridDim.x - 1) / gridDim.x;
    const int64_t r0 = int64_t(blockIdx.x) * chunk, r1 = min(R, r0 + chunk);
    const float* recs = ilql_recs(a);
    // acc: 0 Σ ce·attn (AWAC)  1,2 Σ ce·done per head (CQL)  3,4 Σ td² per head  5 Σ v-loss
    double acc[6] = {0, 0, 0, 0, 0, 0};
    static_assert(kIlqlRec == 4, "one 16-B load per record");
    for (int64_t r = r0 + threadIdx.x; r < r1; r += blockDim.x) {
        const vec4u rv = *reinterpret_cast<const vec4u*>(recs + r * kIlqlRec);
        const float c0 = __uint_as_float(rv.x), c1 = __uint_as_float(rv.y), c2 = __uint_as_float(rv.z);
        if (r < nl) {
            acc[0] += double(c0);
        } else {
            const int h = int((r - nl) / na);
            acc[1 + h] += double(c0);
            acc[3 + h] += double(c1);
            acc[5] += double(c2);
        }
    }
    const double t = block_sum_multi<6>(acc, sh);
    const IlqlRed red = ilql_red(a);
    if (!publish_record_last<6>(red.fin_rec + blockIdx.x * 6, t, red.tickets + 1, gridDim.x)) return;
    __syncthreads();  // sh[] reuse
    const double f = reduce_records<6>(red.fin_rec, int(gridDim.x), sh);
    if (threadIdx.x < 6) tot[threadIdx.x] = f;
    __syncthreads();
    if (threadIdx.x == 0) {
        const double* sums = ilql_sums(a);
        const double n = sums[0], nattn = sums[1];
        const double loss_q = tot[3] / n + tot[4] / n;
        const double loss_v = tot[5] / n;
        const double loss_cql = tot[1] / n + tot[2] / n;
        const double loss_awac = tot[0] / nattn;
        const double loss = loss_q + loss_v + double(a.cql_scale) * loss_cql + double(a.awac_scale) * loss_awac;
        a.losses[0] = float(loss);
        a.losses[1] = float(loss_q);
        a.losses[2] = float(loss_v);
        a.losses[3] = float(loss_cql);
        a.losses[4] = float(loss_awac);
    }
}

// ------------------------------------------------------------------ host side
int tuning_split_lds();  // vocab_rows.hip ("split_lds")
int tuning_ilql_split();  // vocab_rows.hip ("ilql_split")

static const int kIlqlNVs[] = {1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 13, 16};

// Register-resident geometry: the smallest NV that holds the row in <= 512 threads, else
// <= 1024 threads (fp32 V = 50257: 1024 threads x 13 vectors).
static bool ilql_geometry(int64_t V, int elem_bytes, int& nv, int& threads) {
    const int epv = 16 / elem_bytes;
    const int64_t nvec = V / epv + 1 + (kLineVecs - 1);
    for (int pref : {512, kMaxThreads}) {
        const int64_t need = (nvec + pref - 1) / pref;
        for (int c : kIlqlNVs) {
            if (c < need) continue;
            int64_t thr = (nvec + c - 1) / c;
            thr = ((thr + kWave - 1) / kWave) * kWave;
            nv = c;
            threads = int(thr < kWave ? kWave : thr);
            return true;
        }
    }
    return false;
}

static bool same_phase(const void* x, int64_t sb, int64_t st, const void* dx, int64_t dsb, int64_t dst,
                       int64_t B, int64_t T, size_t es) {
    return (B <= 1 || ((sb - dsb) * int64_t(es)) % 16 == 0) && (T <= 1 || ((st - dst) * int64_t(es)) % 16 == 0) &&
           ((reinterpret_cast<uintptr_t>(x) ^ reinterpret_cast<uintptr_t>(dx)) & 15u) == 0;
}

static int ilql_check(const trlx_ilql_args* p) {
    TRLX_REQUIRE(p, TRLX_ERR_ARG, "NULL trlx_ilql_args");
    const trlx_ilql_args& a = *p;
    TRLX_REQUIRE(a.dtype == TRLX_F32 || a.dtype == TRLX_BF16, TRLX_ERR_DTYPE, "ILQL rows dtype %d", a.dtype);
    TRLX_REQUIRE(a.nq == 1 || a.nq == 2, TRLX_ERR_ARG, "nq must be 1 or 2 (got %d)", a.nq);
    TRLX_REQUIRE(a.B > 0 && a.L >= 1 && a.A >= 1 && a.V > 0, TRLX_ERR_SHAPE,
                 "bad ILQL shape B=%lld L=%lld A=%lld V=%lld", (long long)a.B, (long long)a.L, (long long)a.A,
                 (long long)a.V);
    TRLX_REQUIRE(ilql_num_rows(a.B, a.L, a.A, a.nq) <= 0x7fffffffLL, TRLX_ERR_SHAPE, "too many rows");
    TRLX_REQUIRE(a.V * 16 < (1LL << 32), TRLX_ERR_SHAPE, "vocab too large");
    TRLX_REQUIRE(a.logits && a.q[0] && a.tq[0] && (a.nq == 1 || (a.q[1] && a.tq[1])), TRLX_ERR_ARG,
                 "NULL logits / Q-head pointer");
    TRLX_REQUIRE(a.input_ids && a.attention_mask && a.actions_ixs && a.dones && a.rewards && a.vs, TRLX_ERR_ARG,
                 "NULL batch tensor");
    TRLX_REQUIRE(a.dlogits && a.dq[0] && (a.nq == 1 || a.dq[1]) && a.dvs && a.losses && a.workspace,
                 TRLX_ERR_ARG, "NULL output / workspace");
    return TRLX_OK;
}

template <class DT>
static int ilql_launch_rows(const trlx_ilql_args& a, hipStream_t stream) {
    const size_t es = sizeof(typename DT::elem_t);
    TRLX_REQUIRE(same_phase(a.logits, a.logits_sb, a.logits_st, a.dlogits, a.dlogits_sb, a.dlogits_st, a.B, a.L, es),
                 TRLX_ERR_STRIDE, "dlogits rows must have the logits rows' 16-B phase (grad_buffer_like)");
    for (int h = 0; h < a.nq; ++h)
        TRLX_REQUIRE(same_phase(a.q[h], a.q_sb[h], a.q_st[h], a.dq[h], a.dq_sb[h], a.dq_st[h], a.B, a.A, es),
                     TRLX_ERR_STRIDE, "dq rows must have the q rows' 16-B phase (grad_buffer_like)");
    if (es == 4 && tuning_split_lds() != 1) {  // long fp32 rows: split VGPR + LDS residency
        const int64_t nvec = a.V / 4 + 1 + (kLineVecs - 1);
        if (nvec > 512 * 16 && nvec <= 512 * (20 + 5)) {
            const dim3 grid(unsigned(ilql_num_rows(a.B, a.L, a.A, a.nq)));
            switch (tuning_ilql_split()) {
                case 1: hipLaunchKernelGGL((k_ilql_rows<DT, 22, 3>), grid, dim3(512), 0, stream, a); break;
                case 2: hipLaunchKernelGGL((k_ilql_rows<DT, 21, 4>), grid, dim3(512), 0, stream, a); break;
                case 3: hipLaunchKernelGGL((k_ilql_rows<DT, 19, 6>), grid, dim3(512), 0, stream, a); break;
                default: hipLaunchKernelGGL((k_ilql_rows<DT, 20, 5>), grid, dim3(512), 0, stream, a); break;
            }
            return check_launch("k_ilql_rows (split LDS)");
        }
    }
    int nv = 0, thr = 0;
    TRLX_REQUIRE(ilql_geometry(a.V, int(es), nv, thr), TRLX_ERR_SHAPE,
                 "vocab %lld too long for register-resident ILQL rows", (long long)a.V);
    const dim3 grid(unsigned(ilql_num_rows(a.B, a.L, a.A, a.nq))), block(thr);
#define TRLX_ILQL_CASE(N) \
    case N: hipLaunchKernelGGL((k_ilql_rows<DT, N>), grid, block, 0, stream, a); break;
    switch (nv) {
        TRLX_ILQL_CASE(1) TRLX_ILQL_CASE(2) TRLX_ILQL_CASE(3) TRLX_ILQL_CASE(4) TRLX_ILQL_CASE(5)
        TRLX_ILQL_CASE(6) TRLX_ILQL_CASE(7) TRLX_ILQL_CASE(8) TRLX_ILQL_CASE(10) TRLX_ILQL_CASE(12)
        TRLX_ILQL_CASE(13) TRLX_ILQL_CASE(16)
        default: TRLX_REQUIRE(false, TRLX_ERR_SHAPE, "no ILQL geometry for NV=%d", nv);
    }
#undef TRLX_ILQL_CASE
    return check_launch("k_ilql_rows");
}

}  // namespace trlx

using namespace trlx;

extern "C" int64_t trlx_ilql_workspace_bytes(int64_t B, int64_t L, int64_t A, int nq) {
    return ilql_red_offset(ilql_num_rows(B, L, A, nq)) + 16 + int64_t(sizeof(double)) * kIlqlRedMaxBlocks * (2 + 6);
}

extern "C" int trlx_ilql_prep(const trlx_ilql_args* args, void* stream) {
    int rc = ilql_check(args);
    if (rc) return rc;
    const int nblk = ilql_red_blocks(args->B * std::max(args->A, args->L - 1), kIlqlPrepPerBlock);
    hipLaunchKernelGGL(k_ilql_prep, dim3(nblk), dim3(kIlqlRedThreads), 0, (hipStream_t)stream, *args);
    return check_launch("k_ilql_prep");
}

extern "C" int trlx_ilql_rows(const trlx_ilql_args* args, void* stream) {
    int rc = ilql_check(args);
    if (rc) return rc;
    if (args->dtype == TRLX_BF16) return ilql_launch_rows<BF16T>(*args, (hipStream_t)stream);
    return ilql_launch_rows<F32T>(*args, (hipStream_t)stream);
}

extern "C" int trlx_ilql_finalize(const trlx_ilql_args* args, void* stream) {
    int rc = ilql_check(args);
    if (rc) return rc;
    const int nblk = ilql_red_blocks(ilql_num_rows(args->B, args->L, args->A, args->nq), kIlqlFinPerBlock);
    hipLaunchKernelGGL(k_ilql_finalize, dim3(nblk), dim3(kIlqlRedThreads), 0, (hipStream_t)stream, *args);
    return check_launch("k_ilql_finalize");
}

extern "C" int trlx_ilql_loss_fused(const trlx_ilql_args* args, void* stream) {
    int rc = trlx_ilql_prep(args, stream);
    if (rc) return rc;
    rc = trlx_ilql_rows(args, stream);
    if (rc) return rc;
    return trlx_ilql_finalize(args, stream);
}
