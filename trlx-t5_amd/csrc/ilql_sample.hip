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


// phase stamps for tools/smp_probe.hip (never compiled into the library)
#ifdef TRLX_SMP_PROF
__device__ uint64_t g_smp_prof[4096][12];
#define SMP_STAMP(i) \
    if (threadIdx.x == 0) g_smp_prof[blockIdx.x][i] = wall_clock64()
#define SMP_COUNT(i, v) g_smp_prof[blockIdx.x][i] = uint64_t(v)
#else
#define SMP_STAMP(i)
#define SMP_COUNT(i, v)
#endif

// order-preserving float -> uint32 (a larger float has a larger key) and back
__device__ __forceinline__ uint32_t fkey(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float fkey_inv(uint32_t k) {  // NaN for keys no float maps to
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// NT threads per row: 1024 while the row fits in 128 VGPRs per thread, 512 (256 VGPRs per
// thread) for the long rows, which would spill at 1024
constexpr int kCandCap = 512;  // candidate list (scores >= t0) in LDS, one per thread at most

template <class DT, int NV, int NT>
__global__ __launch_bounds__(NT) void k_ilql_sample(SampleArgs a) {
    constexpr int kSmpThreads = NT;
    constexpr int kSmpWaves = NT / kWave;
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
    __shared__ float t_max[kSmpThreads];     // per-thread maximum score
    __shared__ __align__(16) float c_val[kCandCap + 4];  // candidates: every score >= t0
    __shared__ __align__(16) float c_w[kCandCap + 4];    // their weights
    __shared__ __align__(16) int c_idx[kCandCap + 4];
    __shared__ int c_n;
    __shared__ float s_thr;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int b = blockIdx.x;
    const int64_t V = a.V;
    if (a.finished && a.finished[b]) {  // (1 - finished) * ids + finished * eos: the draw is unused
        if (tid == 0) a.out_ids[b] = a.eos;
        return;
    }

    const E* x = reinterpret_cast<const E*>(a.logits) + b * a.ld_logits;
    const RowSplit<DT> s(x, V);
    const int nvec = int(s.nvec);
    const int shift = line_shift(x + s.head);
    const int voff = (tid - shift) * 16;
    const uint8_t* mrow = a.logit_mask ? a.logit_mask + a.prev_ids[b] * a.ld_mask : nullptr;
    const __amdgpu_buffer_rsrc_t rin = make_rsrc(x + s.head, uint32_t(nvec) * 16u);
    auto valid = [&](int k) { return unsigned(tid - shift + k * kSmpThreads) < unsigned(nvec); };
    // recomputed at every use (laundered): CSE would keep NV 64-bit indices live across the kernel
    auto index_of = [&](int k, int e) {
        return s.head + int64_t(launder_int(tid - shift) + k * kSmpThreads) * EPV + e;
    };

    SMP_STAMP(0);
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

    SMP_STAMP(1);
    // ---- log_softmax statistics (F.log_softmax(logits, -1)): exponentials relative to the
    // wave maximum, then one exchange of (wave max, wave sum) pairs — one barrier
    float m = fe;
#pragma unroll
    for (int k = 0; k < NV; ++k)
#pragma unroll
        for (int e = 0; e < EPV; ++e) m = fmaxf(m, f[k][e]);
    m = wave_max(m);
    // exp2(-inf) = 0 for masked entries; a wave with nothing but -inf contributes nothing
    const float mo = m == -INFINITY ? 0.f : m * kLog2e;
    float sum = exp2_fast(__builtin_fmaf(fe, kLog2e, -mo));
#pragma unroll
    for (int k = 0; k < NV; ++k)
#pragma unroll
        for (int e = 0; e < EPV; ++e) sum += exp2_fast(__builtin_fmaf(f[k][e], kLog2e, -mo));
    sum = wave_sum(sum);
    if (lane == 0) {
        sh_red[wv] = m;
        sh_red2[wv] = sum;
    }
    __syncthreads();
    m = sh_red[0];
#pragma unroll
    for (int w = 1; w < kSmpWaves; ++w) m = fmaxf(m, sh_red[w]);
    sum = 0.f;
#pragma unroll
    for (int w = 0; w < kSmpWaves; ++w)
        if (sh_red[w] != -INFINITY) sum += sh_red2[w] * exp2_fast((sh_red[w] - m) * kLog2e);
    const float lse = m + logf(sum);

    SMP_STAMP(2);
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
            // a window of kQWin vector steps in flight; the scheduling fences keep the
            // compiler from hoisting every load to the top (3x the row in VGPRs -> spills)
            constexpr int kQWin = NV < 4 ? NV : 4;
            vec4u w0[kQWin], w1[kQWin];
#pragma unroll
            for (int k = 0; k < kQWin; ++k) {
                w0[k] = __builtin_amdgcn_raw_buffer_load_b128(r0, launder_int(voff) + k * kSmpThreads * 16, 0, kAuxNT);
                w1[k] = __builtin_amdgcn_raw_buffer_load_b128(r1, launder_int(voff) + k * kSmpThreads * 16, 0, kAuxNT);
            }
#pragma unroll
            for (int k = 0; k < NV; ++k) {
                float t0[EPV], t1[EPV];
                DT::unpack(w0[k % kQWin], t0);
                DT::unpack(w1[k % kQWin], t1);
                if (k + kQWin < NV) {
                    const int o = launder_int(voff) + (k + kQWin) * kSmpThreads * 16;
                    w0[k % kQWin] = __builtin_amdgcn_raw_buffer_load_b128(r0, o, 0, kAuxNT);
                    w1[k % kQWin] = __builtin_amdgcn_raw_buffer_load_b128(r1, o, 0, kAuxNT);
                }
#pragma unroll
                for (int e = 0; e < EPV; ++e)  // -inf stays -inf (masked / out-of-row slots)
                    f[k][e] = add_rn(f[k][e] - lse, mul_rn(a.beta, fminf(t0[e], t1[e]) - vsb));
                __builtin_amdgcn_sched_barrier(0);
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

    SMP_STAMP(3);
    // (from here on a slot outside the row or masked holds -inf, which no count or weight
    // below can pick: no per-slot validity test is needed)
    // ---- the k-th largest score: bisection on the order-preserving keys, MSB first — the
    // largest key K with #(key >= K) >= k IS the k-th largest key.  One block-wide count per
    // bit (compares + a wave sum + one LDS exchange; no atomics: the scores crowd a few
    // exponent values, which would serialise histogram atomics on a handful of bins).
    float thr = -INFINITY;  // keep !(score < thr); top_k > V keeps everything (topk_mask)
    int mode = 0;           // 1: wave 0 drew the token from the candidate list
    if (int64_t(a.top_k) <= V) {
        // Candidate pre-filter: t0 = the k-th largest of the per-thread maxima is a lower
        // bound of the k-th largest score (k threads each own a score >= t0), so the scores
        // >= t0 — a few times k on real rows — hold the whole top-k set.  They are appended
        // to LDS; the exact threshold and the draw then run in one wave without barriers.
        // Rows that defeat the filter (ties, -inf-heavy rows, k > threads) take the
        // block-wide bisection over all scores below.
        bool cands = false;
        if (a.top_k <= kSmpThreads) {
            float mx = je >= 0 ? fe : -INFINITY;
#pragma unroll
            for (int k = 0; k < NV; ++k)
#pragma unroll
                for (int e = 0; e < EPV; ++e) mx = fmaxf(mx, f[k][e]);
            t_max[tid] = mx;
            if (tid == 0) {
                c_n = 0;
                s_pick[2] = -1;
            }
            __syncthreads();
            if (wv == 0) {
                constexpr int R = kSmpThreads / kWave;
                float tv[R];
#pragma unroll
                for (int i = 0; i < R; ++i) tv[i] = t_max[lane + i * kWave];
                // the top 16 key bits (sign, exponent, 7 mantissa bits) are enough for a
                // lower bound: K <= the exact key, a few more candidates at most
                uint32_t K = 0;
                for (int bit = 31; bit >= 16; --bit) {
                    const uint32_t cand = K | (1u << bit);
                    const float cf = fkey_inv(cand);
                    int c = 0;
#pragma unroll
                    for (int i = 0; i < R; ++i) c += __popcll(__ballot(tv[i] >= cf));
                    if (c >= a.top_k) K = cand;
                }
                if (lane == 0) s_thr = K >= fkey(-INFINITY) ? fkey_inv(K) : -INFINITY;
            }
            __syncthreads();
            SMP_STAMP(7);
            const float t0 = s_thr;
            if (t0 != -INFINITY) {
                auto append = [&](bool p, int64_t j, float v) {
                    const uint64_t m = __ballot(p);
                    if (m == 0) return;
                    const int leader = __ffsll((unsigned long long)m) - 1;
                    int base = 0;
                    if (lane == leader) base = atomicAdd(&c_n, __popcll(m));
                    base = __shfl(base, leader, kWave);
                    const int pos = base + __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32),
                                                                     __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0));
                    if (p && pos < kCandCap) {
                        c_val[pos] = v;
                        c_idx[pos] = int(j);
                    }
                };
                append(je >= 0 && fe >= t0, je, fe);
#pragma unroll
                for (int k = 0; k < NV; ++k)
#pragma unroll
                    for (int e = 0; e < EPV; ++e) append(f[k][e] >= t0, index_of(k, e), f[k][e]);
            }
            __syncthreads();
            SMP_STAMP(8);
            if (threadIdx.x == 0) SMP_COUNT(9, c_n);
            cands = t0 != -INFINITY && c_n <= kCandCap;  // block-uniform
        }
        if (cands) {
            // every thread ranks at most one candidate against the whole list (LDS broadcast
            // reads): the k-th largest is the value with #(>) < k <= #(>=) — exact, with ties
            const int n = c_n;
            if (tid < 4) {  // pad to whole float4s: -inf and zero weights never count
                c_val[n + tid] = -INFINITY;
                c_w[n + tid] = 0.f;
                c_idx[n + tid] = INT_MAX;
            }
            __syncthreads();
            const bool own = tid < n;
            const float vt = own ? c_val[tid] : -INFINITY;
            const int jt = own ? c_idx[tid] : 0;
            int gt = 0, ge = 0;
            float vmax = -INFINITY;
            for (int q = 0; q < n; q += 4) {
                const float4 vq = *reinterpret_cast<const float4*>(&c_val[q]);
                gt += (vq.x > vt) + (vq.y > vt) + (vq.z > vt) + (vq.w > vt);
                ge += (vq.x >= vt) + (vq.y >= vt) + (vq.z >= vt) + (vq.w >= vt);
                vmax = fmaxf(fmaxf(vmax, fmaxf(vq.x, vq.y)), fmaxf(vq.z, vq.w));
            }
            if (own && gt < a.top_k && a.top_k <= ge) s_thr = vt;  // every writer holds the same value
            __syncthreads();
            thr = s_thr;
            // softmax(kept / T) — max(v / T) = max(v) / T: division by T > 0 is monotone — and
            // the inverse CDF at u in index order: a kept entry's interval starts at the sum
            // of the kept weights with a smaller vocab index
            const float T = a.temperature;
            const float zmax = vmax / T;
            const float wt = (own && !(vt < thr)) ? exp2_fast((vt / T - zmax) * kLog2e) : 0.f;
            if (own) c_w[tid] = wt;
            __syncthreads();
            float pre = 0.f, tot = 0.f;
            for (int q = 0; q < n; q += 4) {
                const float4 wq = *reinterpret_cast<const float4*>(&c_w[q]);
                const int4 jq = *reinterpret_cast<const int4*>(&c_idx[q]);
                tot += wq.x + wq.y + wq.z + wq.w;
                pre += (jq.x < jt ? wq.x : 0.f) + (jq.y < jt ? wq.y : 0.f) + (jq.z < jt ? wq.z : 0.f) +
                       (jq.w < jt ? wq.w : 0.f);
            }
            // the kept entry with the largest index whose interval starts at or below the target
            if (wt > 0.f && pre <= a.u[b] * tot) atomicMax(&s_pick[2], jt);
            mode = 1;
        } else {
            // block-wide bisection over every score, MSB first: the largest K with
            // #(key >= K) >= k IS the k-th largest key.  One count per bit (compares + a
            // wave sum + one LDS exchange; no atomics: the scores crowd a few exponent
            // values, which would serialise histogram atomics on a handful of bins).  The
            // candidate is turned into a float, not every score into a key: one compare
            // per element per bit.  Float >= is monotone in the key; candidates in the NaN
            // key ranges count 0, so K never lands there.
            uint32_t K = 0;
            for (int bit = 31; bit >= 0; --bit) {
                const uint32_t cand = K | (1u << bit);
                const float cf = fkey_inv(cand);
                int c = (je >= 0 && fe >= cf) ? 1 : 0;
#pragma unroll
                for (int k = 0; k < NV; ++k)
#pragma unroll
                    for (int e = 0; e < EPV; ++e) c += f[k][e] >= cf ? 1 : 0;
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, kWave);
                if (lane == 0) cnt[bit & 1][wv] = c;
                __syncthreads();  // double-buffered counts: one barrier per bit
                int tot = 0;
#pragma unroll
                for (int w = 0; w < kSmpWaves; ++w) tot += cnt[bit & 1][w];
                if (tot >= a.top_k) K = cand;
            }
            // fewer than k finite scores: K stays below the key of -inf, everything finite is kept
            thr = K >= fkey(-INFINITY) ? fkey_inv(K) : -INFINITY;
        }
    }

    SMP_STAMP(4);
    if (mode == 0) {
    // ---- weights exp(score / T - max) of the kept entries
    const float T = a.temperature;
    auto kept = [&](float v, bool ok) { return ok && !(v < thr) && v != -INFINITY; };
    float zmax = kept(fe, je >= 0) ? fe / T : -INFINITY;
#pragma unroll
    for (int k = 0; k < NV; ++k)
#pragma unroll
        for (int e = 0; e < EPV; ++e)
            if (kept(f[k][e], true)) zmax = fmaxf(zmax, f[k][e] / T);
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
            const float w = kept(f[k][e], true) ? exp2_fast((f[k][e] / T - zmax) * kLog2e) : 0.f;
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

    SMP_STAMP(5);
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
    }  // mode == 0
    __syncthreads();
    SMP_STAMP(6);
    if (tid == 0) {
        const int64_t tok = s_pick[2] < 0 ? 0 : s_pick[2];  // nothing kept: torch.multinomial would raise
        a.out_ids[b] = tok;  // (finished rows returned eos at the top)
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
    auto need = [&](int nt) { return (V / epv + 1 + (kLineVecs - 1) + nt - 1) / nt; };  // vectors per thread
#define TRLX_SMP(DTT, N, NT)                                                                              \
    if (need(NT) <= N) {                                                                                  \
        hipLaunchKernelGGL((k_ilql_sample<DTT, N, NT>), dim3(unsigned(B)), dim3(NT), 0, (hipStream_t)stream, a); \
        return check_launch("k_ilql_sample");                                                             \
    }
    if (dtype == TRLX_BF16) {
        TRLX_SMP(BF16T, 1, 1024)
        TRLX_SMP(BF16T, 4, 1024)
        TRLX_SMP(BF16T, 8, 512)
        TRLX_SMP(BF16T, 13, 512)
        TRLX_SMP(BF16T, 16, 512)
        TRLX_SMP(BF16T, 16, 1024)
    } else {
        TRLX_SMP(F32T, 1, 1024)
        TRLX_SMP(F32T, 4, 1024)
        TRLX_SMP(F32T, 8, 1024)
        TRLX_SMP(F32T, 16, 512)
        TRLX_SMP(F32T, 26, 512)
        TRLX_SMP(F32T, 32, 512)
    }
#undef TRLX_SMP
    TRLX_REQUIRE(false, TRLX_ERR_SHAPE, "vocab %lld too long for the sampling kernel", (long long)V);
}
