// Vocab-axis sampling step of ILQL generation, one workgroup per row:
// CausalLMWithValueHeads.generate, trlx/model/nn/ilql_models.py:296-316, with topk_mask
// (:24-28, = trlx/utils/__init__.py:107-116):
//
//   x      = logits[b, -1, :]  (-inf where logit_mask[input_ids[b, -1]] is set)
//   score  = log_softmax(x) + beta * (min_i target_q_i[b, -1, :] - vs[b, -1])
//   keep   = !(score < k-th largest score)        (topk_mask: ties at the threshold kept)
//   pi     = softmax(where(keep, score, -inf) / temperature)
//   token  = inverse CDF of pi at u[b], index order   (the torch.multinomial draw)
//   token  = finished ? eos : token;  finished = token == eos
//
// The logits row is held in VGPRs (16-B buffer loads on the rows' 256-B line shift), the
// target-Q rows stream through once; the k-th largest score is a 32-step bisection over
// order-preserving uint32 keys (block-wide counts); the draw is a prefix over
// the kept exponentials in index order (segment totals, then a wave scan inside the
// segment).  HBM: (1 + nq) row reads per sampled token; latency-bound at decode batch sizes.
#include "common.h"

namespace trlx {

struct SampleArgs {
    const void* logits;      // [B, V] rows of ld_logits
    int64_t ld_logits;
    const void* tq[2];       // target-Q heads [B, V]
    int64_t ld_tq[2];
    int nq;
    const float* vs;         // [B] state values V(s_t)
    const uint8_t* logit_mask;  // NULL or [Vm, V] bool rows, row chosen by prev_ids[b]
    int64_t ld_mask;
    const int64_t* prev_ids;    // [B] last input token (row of logit_mask)
    int64_t V;
    float beta, temperature;
    int top_k;
    const float* u;          // [B] uniforms in [0, 1)
    int64_t* out_ids;        // [B]
    int64_t* finished;       // [B] in/out (0/1), NULL = none finished
    int64_t eos;
};

constexpr int kSmpThreads = 1024;
constexpr int kSmpWaves = kSmpThreads / kWave;

// order-preserving float -> uint32 (a larger float has a larger key) and back
__device__ __forceinline__ uint32_t fkey(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float fkey_inv(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

template <class DT, int NV>
__global__ __launch_bounds__(kSmpThreads) void k_ilql_sample(SampleArgs a) {
    typedef typename DT::elem_t E;
    constexpr int EPV = DT::kEPV;
    constexpr int NSEG = NV + 2;  // index-order segments: head elements, vector steps, tail
    __shared__ float sh_red[kSmpWaves];
    __shared__ float sh_red2[kSmpWaves];
    __shared__ float sh_red3[kSmpWaves];
    __shared__ int cnt[2][kSmpWaves];        // bisection counts (double-buffered)
    __shared__ float seg_tot[NSEG][kSmpWaves];
    __shared__ float seg_pre[NSEG + 1];
    __shared__ int s_pick[3];                // segment, winning thread, token
    __shared__ float s_rem;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int b = blockIdx.x;
    const int64_t V = a.V;

    const E* x = reinterpret_cast<const E*>(a.logits) + b * a.ld_logits;
    const RowSplit<DT> s(x, V);
    const int nvec = int(s.nvec);
    const int shift = line_shift(x + s.head);
    const int voff = (tid - shift) * 16;
    const uint8_t* mrow = a.logit_mask ? a.logit_mask + a.prev_ids[b] * a.ld_mask : nullptr;
    const __amdgpu_buffer_rsrc_t rin = make_rsrc(x + s.head, uint32_t(nvec) * 16u);
    auto valid = [&](int k) { return unsigned(tid - shift + k * kSmpThreads) < unsigned(nvec); };
    auto index_of = [&](int k, int e) { return s.head + int64_t(tid - shift + k * kSmpThreads) * EPV + e; };

    // ---- logits row -> registers (masked / out-of-row entries -inf); <= 1 edge element per thread
    float f[NV][EPV];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const vec4u v = __builtin_amdgcn_raw_buffer_load_b128(rin, launder_int(voff) + k * kSmpThreads * 16, 0, kAuxNT);
        DT::unpack(v, f[k]);
    }
    int64_t je = -1;  // head element -> threads [0, head); tail -> the last `tail` threads
    if (tid < s.head) je = tid;
    else if (tid >= kSmpThreads - s.tail) je = s.tail0 + (tid - (kSmpThreads - s.tail));
    float fe = je >= 0 ? DT::load1(x, je) : -INFINITY;
#pragma unroll
    for (int k = 0; k < NV; ++k)
#pragma unroll
        for (int e = 0; e < EPV; ++e) {
            bool dead = !valid(k);
            if (!dead && mrow) dead = mrow[index_of(k, e)] != 0;
            if (dead) f[k][e] = -INFINITY;
        }
    if (je >= 0 && mrow && mrow[je]) fe = -INFINITY;

    // ---- log_softmax statistics (F.log_softmax(logits, -1))
    float m = fe;
#pragma unroll
    for (int k = 0; k < NV; ++k)
#pragma unroll
        for (int e = 0; e < EPV; ++e) m = fmaxf(m, f[k][e]);
    m = block_max(m, sh_red);
    float sum = fe == -INFINITY ? 0.f : exp2_fast((fe - m) * kLog2e);
#pragma unroll
    for (int k = 0; k < NV; ++k)
#pragma unroll
        for (int e = 0; e < EPV; ++e) sum += f[k][e] == -INFINITY ? 0.f : exp2_fast((f[k][e] - m) * kLog2e);
    sum = block_sum(sum, sh_red2);
    const float lse = m + logf(sum);

    // ---- score = log_softmax + beta * (min_i tq_i - vs)   (target-Q rows streamed once)
    const float vsb = a.vs[b];
    {
        const E* q0 = reinterpret_cast<const E*>(a.tq[0]) + b * a.ld_tq[0];
        const E* q1 = reinterpret_cast<const E*>(a.tq[a.nq > 1 ? 1 : 0]) + b * a.ld_tq[a.nq > 1 ? 1 : 0];
        const uintptr_t xp = reinterpret_cast<uintptr_t>(x);
        if (((reinterpret_cast<uintptr_t>(q0) ^ xp) & 15u) == 0 && ((reinterpret_cast<uintptr_t>(q1) ^ xp) & 15u) == 0) {
            // same 16-B phase as the logits row (heads of one model output): the same vectors
            const __amdgpu_buffer_rsrc_t r0 = make_rsrc(q0 + s.head, uint32_t(nvec) * 16u);
            const __amdgpu_buffer_rsrc_t r1 = make_rsrc(q1 + s.head, uint32_t(nvec) * 16u);
#pragma unroll
            for (int k = 0; k < NV; ++k) {
                float t0[EPV], t1[EPV];
                DT::unpack(__builtin_amdgcn_raw_buffer_load_b128(r0, launder_int(voff) + k * kSmpThreads * 16, 0,
                                                                 kAuxNT), t0);
                DT::unpack(__builtin_amdgcn_raw_buffer_load_b128(r1, launder_int(voff) + k * kSmpThreads * 16, 0,
                                                                 kAuxNT), t1);
#pragma unroll
                for (int e = 0; e < EPV; ++e)
                    f[k][e] = add_rn(f[k][e] - lse, mul_rn(a.beta, fminf(t0[e], t1[e]) - vsb));
            }
        } else {
#pragma unroll
            for (int k = 0; k < NV; ++k) {
                if (!valid(k)) continue;
                const int64_t j0 = index_of(k, 0);
#pragma unroll
                for (int e = 0; e < EPV; ++e) {
                    const float qm = fminf(DT::load1(q0, j0 + e), DT::load1(q1, j0 + e));
                    f[k][e] = add_rn(f[k][e] - lse, mul_rn(a.beta, qm - vsb));
                }
            }
        }
        if (je >= 0) fe = add_rn(fe - lse, mul_rn(a.beta, fminf(DT::load1(q0, je), DT::load1(q1, je)) - vsb));
    }

    // ---- the k-th largest score: bisection on the order-preserving keys, MSB first — the
    // largest key K with #(key >= K) >= k IS the k-th largest key.  One block-wide count per
    // bit (compares + a wave sum + one LDS exchange; no atomics: the scores crowd a few
    // exponent values, which would serialise histogram atomics on a handful of bins).
    float thr = -INFINITY;  // keep !(score < thr); top_k > V keeps everything (topk_mask)
    if (int64_t(a.top_k) <= V) {
        uint32_t K = 0;
        for (int bit = 31; bit >= 0; --bit) {
            const uint32_t cand = K | (1u << bit);
            int c = (je >= 0 && fkey(fe) >= cand) ? 1 : 0;
#pragma unroll
            for (int k = 0; k < NV; ++k)
#pragma unroll
                for (int e = 0; e < EPV; ++e) c += (valid(k) && fkey(f[k][e]) >= cand) ? 1 : 0;
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, kWave);
            if (lane == 0) cnt[bit & 1][wv] = c;
            __syncthreads();  // double-buffered counts: one barrier per bit
            int tot = 0;
#pragma unroll
            for (int w = 0; w < kSmpWaves; ++w) tot += cnt[bit & 1][w];
            if (tot >= a.top_k) K = cand;
        }
        thr = fkey_inv(K);
    }

    // ---- weights exp(score / T - max) of the kept entries
    const float T = a.temperature;
    auto kept = [&](float v, bool ok) { return ok && !(v < thr) && v != -INFINITY; };
    float zmax = kept(fe, je >= 0) ? fe / T : -INFINITY;
#pragma unroll
    for (int k = 0; k < NV; ++k)
#pragma unroll
        for (int e = 0; e < EPV; ++e)
            if (kept(f[k][e], valid(k))) zmax = fmaxf(zmax, f[k][e] / T);
    zmax = block_max(zmax, sh_red3);
    const float ew = (je >= 0 && kept(fe, true)) ? exp2_fast((fe / T - zmax) * kLog2e) : 0.f;
    const int eseg = je < s.head ? 0 : NSEG - 1;  // the edge element's segment
    // the registers now hold the unnormalised probabilities; per-wave segment totals go
    // straight to LDS (no per-thread segment array: it would spill at 1024 threads)
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        float t = 0.f;
#pragma unroll
        for (int e = 0; e < EPV; ++e) {
            const float w = kept(f[k][e], valid(k)) ? exp2_fast((f[k][e] / T - zmax) * kLog2e) : 0.f;
            f[k][e] = w;
            t += w;
        }
        t = wave_sum(t);
        if (lane == 0) seg_tot[1 + k][wv] = t;
    }
    {
        const float t0 = wave_sum(eseg == 0 ? ew : 0.f), t1 = wave_sum(eseg == 0 ? 0.f : ew);
        if (lane == 0) {
            seg_tot[0][wv] = t0;
            seg_tot[NSEG - 1][wv] = t1;
        }
    }

    // ---- inverse CDF at u: segment totals (fixed order) -> segment -> thread -> element
    __syncthreads();
    if (tid == 0) {
        float acc = 0.f;
        for (int g = 0; g < NSEG; ++g) {
            seg_pre[g] = acc;
            for (int w = 0; w < kSmpWaves; ++w) acc += seg_tot[g][w];
        }
        seg_pre[NSEG] = acc;
        const float target = a.u[b] * acc;
        int gsel = -1;
        for (int g = 0; g < NSEG; ++g)
            if (gsel < 0 && seg_pre[g + 1] > target) gsel = g;
        for (int g = NSEG - 1; gsel < 0 && g >= 0; --g)  // rounding at the top: last non-empty
            if (seg_pre[g + 1] > seg_pre[g]) gsel = g;
        s_pick[0] = gsel;
        s_pick[1] = -1;
        s_pick[2] = -1;
        s_rem = gsel < 0 ? 0.f : target - seg_pre[gsel];
    }
    __syncthreads();
    const int gsel = s_pick[0];
    const float rem = s_rem;
    float mine = 0.f, lo = 0.f;
    if (gsel >= 0) {
        if (gsel == 0 || gsel == NSEG - 1) {
            mine = (je >= 0 && eseg == gsel) ? ew : 0.f;
        } else {
#pragma unroll
            for (int k = 0; k < NV; ++k) {
                float t = 0.f;
#pragma unroll
                for (int e = 0; e < EPV; ++e) t += f[k][e];
                mine = k + 1 == gsel ? t : mine;
            }
        }
        float incl = mine;  // exclusive prefix of this thread's share inside the segment
#pragma unroll
        for (int off = 1; off < kWave; off <<= 1) {
            const float y = __shfl_up(incl, off, kWave);
            if (lane >= off) incl += y;
        }
        float woff = 0.f;
        for (int w = 0; w < wv; ++w) woff += seg_tot[gsel][w];
        lo = woff + incl - mine;
        // the last thread (index order) whose share starts at or below the target
        if (mine > 0.f && lo <= rem) atomicMax(&s_pick[1], tid);
    }
    __syncthreads();
    if (gsel >= 0 && tid == s_pick[1]) {
        int64_t pick = -1;
        if (gsel == 0 || gsel == NSEG - 1) {
            pick = je;
        } else {
            float run = lo;
#pragma unroll
            for (int k = 0; k < NV; ++k) {
                if (k + 1 != gsel) continue;
#pragma unroll
                for (int e = 0; e < EPV; ++e) {
                    if (f[k][e] > 0.f && (pick < 0 || run <= rem)) {
                        pick = index_of(k, e);
                        run += f[k][e];
                        if (run > rem) run = INFINITY;  // found: later elements keep the pick
                    }
                }
            }
        }
        s_pick[2] = int(pick);
    }
    __syncthreads();
    if (tid == 0) {
        int64_t tok = s_pick[2] < 0 ? 0 : s_pick[2];  // nothing kept: torch.multinomial would raise
        const int64_t fin = a.finished ? a.finished[b] : 0;
        tok = fin ? a.eos : tok;  // (1 - finished) * ids + finished * eos
        a.out_ids[b] = tok;
        if (a.finished) a.finished[b] = tok == a.eos ? 1 : 0;
    }
}

}  // namespace trlx

using namespace trlx;

extern "C" int trlx_ilql_sample(const void* logits, int64_t ld_logits, const void* tq0, int64_t ld_tq0,
                                const void* tq1, int64_t ld_tq1, int dtype, const float* vs,
                                const uint8_t* logit_mask, int64_t ld_mask, const int64_t* prev_ids, int64_t B,
                                int64_t V, float beta, int top_k, float temperature, const float* u,
                                int64_t* out_ids, int64_t* finished, int64_t eos, void* stream) {
    TRLX_REQUIRE(logits && tq0 && vs && u && out_ids, TRLX_ERR_ARG, "NULL argument to trlx_ilql_sample");
    TRLX_REQUIRE(!logit_mask || prev_ids, TRLX_ERR_ARG, "logit_mask needs prev_ids");
    TRLX_REQUIRE(dtype == TRLX_F32 || dtype == TRLX_BF16, TRLX_ERR_DTYPE, "dtype %d", dtype);
    TRLX_REQUIRE(B >= 0 && V > 0 && top_k > 0 && temperature > 0.f, TRLX_ERR_SHAPE, "bad sampling arguments");
    TRLX_REQUIRE(B < (int64_t(1) << 31) && V * 16 < (int64_t(1) << 32), TRLX_ERR_SHAPE, "too large");
    if (B == 0) return TRLX_OK;
    SampleArgs a = {};
    a.logits = logits;
    a.ld_logits = ld_logits;
    a.tq[0] = tq0;
    a.tq[1] = tq1 ? tq1 : tq0;
    a.ld_tq[0] = ld_tq0;
    a.ld_tq[1] = tq1 ? ld_tq1 : ld_tq0;
    a.nq = tq1 ? 2 : 1;
    a.vs = vs;
    a.logit_mask = logit_mask;
    a.ld_mask = ld_mask;
    a.prev_ids = prev_ids;
    a.V = V;
    a.beta = beta;
    a.temperature = temperature;
    a.top_k = top_k;
    a.u = u;
    a.out_ids = out_ids;
    a.finished = finished;
    a.eos = eos;
    const int epv = dtype == TRLX_BF16 ? 8 : 4;
    const int64_t need = (V / epv + 1 + (kLineVecs - 1) + kSmpThreads - 1) / kSmpThreads;  // vectors per thread
#define TRLX_SMP(N)                                                                                       \
    if (need <= N) {                                                                                      \
        if (dtype == TRLX_BF16)                                                                           \
            hipLaunchKernelGGL((k_ilql_sample<BF16T, N>), dim3(unsigned(B)), dim3(kSmpThreads), 0,         \
                               (hipStream_t)stream, a);                                                   \
        else                                                                                              \
            hipLaunchKernelGGL((k_ilql_sample<F32T, N>), dim3(unsigned(B)), dim3(kSmpThreads), 0,          \
                               (hipStream_t)stream, a);                                                   \
        return check_launch("k_ilql_sample");                                                             \
    }
    TRLX_SMP(1)
    TRLX_SMP(4)
    TRLX_SMP(8)
    TRLX_SMP(13)
    TRLX_SMP(16)
#undef TRLX_SMP
    TRLX_REQUIRE(false, TRLX_ERR_SHAPE, "vocab %lld too long for the sampling kernel", (long long)V);
}
