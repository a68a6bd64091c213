// Shared device helpers for the trlx_t5_amd HIP kernels (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "trlx_t5_amd.h"

namespace trlx {

// A launch-geometry knob (trlx_set_tuning): one process-wide value, read by whichever host
// thread launches (PyTorch runs backward nodes on its autograd device thread, so a
// thread-local knob set by the caller would not reach them).
struct TuneKnob {
    int v;
    operator int() const { return __atomic_load_n(&v, __ATOMIC_RELAXED); }
    TuneKnob& operator=(int x) {
        __atomic_store_n(&v, x, __ATOMIC_RELAXED);
        return *this;
    }
};

constexpr int kWave = 64;          // CDNA wavefront
constexpr int kMaxThreads = 1024;  // largest workgroup we launch
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef uint32_t vec4u __attribute__((ext_vector_type(4)));  // one 16-byte row vector
__device__ __forceinline__ vec4u vec4u_make(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    vec4u r = {a, b, c, d};
    return r;
}

// ------------------------------------------------------------------ bf16 <-> f32
__device__ __forceinline__ float bf_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float(uint32_t(h) << 16); }
// round-to-nearest-even, NaN preserving (lowers to v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t pack_bf2(float a, float b) {
    bf16x2_t r;
    r.x = (__bf16)a;
    r.y = (__bf16)b;
    return __builtin_bit_cast(uint32_t, r);
}
__device__ __forceinline__ uint16_t f2bf(float a) {
    __bf16 h = (__bf16)a;
    return __builtin_bit_cast(uint16_t, h);
}

// scalar load / store of a [n] vector of either dtype
__device__ __forceinline__ float ld_any(const void* p, int dtype, int64_t i) {
    return dtype == TRLX_BF16 ? bf2f(reinterpret_cast<const uint16_t*>(p)[i])
                              : reinterpret_cast<const float*>(p)[i];
}
__device__ __forceinline__ void st_any(void* p, int dtype, int64_t i, float v) {
    if (dtype == TRLX_BF16)
        reinterpret_cast<uint16_t*>(p)[i] = f2bf(v);
    else
        reinterpret_cast<float*>(p)[i] = v;
}

// ------------------------------------------------------------------ fast transcendentals
// v_exp_f32 computes 2^x; callers pre-scale by log2(e) (folded into an fma).
__device__ __forceinline__ float exp2_fast(float x) { return __builtin_amdgcn_exp2f(x); }

// Packed-fp32 helpers (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 work on two fp32 lanes per
// instruction at the issue cost of one): the vocab-row passes scale and accumulate element
// pairs with them, leaving one v_exp_f32 per element.  Measured on the C2 experience rows:
// the per-element VALU work (unpack, scale, exp, accumulate) kept the SIMDs ~70 % busy, so
// halving the scale / accumulate instructions shortens the rows at full bandwidth.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 f2_splat(float v) { return f32x2{v, v}; }
__device__ __forceinline__ f32x2 f2_exp2(f32x2 y) { return f32x2{exp2_fast(y.x), exp2_fast(y.y)}; }
__device__ __forceinline__ f32x2 f2_fma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
// Σ over one vector's elements of 2^(f·log2e + c) as a lane pair (element 2i -> .x, 2i+1 -> .y)
template <int N>
__device__ __forceinline__ f32x2 exp_pair_sum(const float (&f)[N], f32x2 l2e, f32x2 c) {
    static_assert(N % 2 == 0, "pairs");
    f32x2 s = f2_exp2(f2_fma(f32x2{f[0], f[1]}, l2e, c));
#pragma unroll
    for (int e = 2; e < N; e += 2) s += f2_exp2(f2_fma(f32x2{f[e], f[e + 1]}, l2e, c));
    return s;
}
// f[e] <- -g · 2^(f[e]·log2e + c) in place (the softmax part of a gradient row)
template <int N>
__device__ __forceinline__ void neg_g_exp_pairs(float (&f)[N], f32x2 l2e, f32x2 c, f32x2 neg_g) {
#pragma unroll
    for (int e = 0; e < N; e += 2) {
        const f32x2 r = neg_g * f2_exp2(f2_fma(f32x2{f[e], f[e + 1]}, l2e, c));
        f[e] = r.x;
        f[e + 1] = r.y;
    }
}

// Two signed 16-bit maxima per instruction (v_pk_max_i16).  Inline asm: hipcc 7.2 folds
// __builtin_elementwise_max over bit-cast short2 vectors of one dwordx4 down to a single dword
// (observed in the ISA), so the builtin is not used.
__device__ __forceinline__ uint32_t pk_max_i16(uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_pk_max_i16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// IEEE ops that must not be contracted into fma (the reference evaluates them as
// separately rounded torch ops).
__device__ __forceinline__ float add_rn(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ float mul_rn(float a, float b) { return __fmul_rn(a, b); }

// ------------------------------------------------------------------ wave / block reductions
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
    return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
    return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
    return v;
}

// Block reductions over blockDim.x (multiple of 64, <= 1024) threads.  `sh` must hold
// blockDim.x/64 slots and be private to this call site (no trailing barrier: every
// thread reads all slots after the one barrier, so a later reduction must use its own
// slots).  The cross-wave order is fixed => deterministic.
__device__ __forceinline__ float block_max(float v, float* sh) {
    v = wave_max(v);
    const int nw = blockDim.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == 0) sh[threadIdx.x / kWave] = v;
    __syncthreads();
    float r = sh[0];
    for (int i = 1; i < nw; ++i) r = fmaxf(r, sh[i]);
    return r;
}
__device__ __forceinline__ float block_sum(float v, float* sh) {
    v = wave_sum(v);
    const int nw = blockDim.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == 0) sh[threadIdx.x / kWave] = v;
    __syncthreads();
    float r = sh[0];
    for (int i = 1; i < nw; ++i) r += sh[i];
    return r;
}
__device__ __forceinline__ double block_sum_d(double v, double* sh) {
    v = wave_sum_d(v);
    const int nw = blockDim.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == 0) sh[threadIdx.x / kWave] = v;
    __syncthreads();
    double r = sh[0];
    for (int i = 1; i < nw; ++i) r += sh[i];
    return r;
}

// K independent fp64 sums over the block with ONE barrier: shuffle-reduce inside each
// wave (the K chains interleave), lane 0 of each wave parks its K sums in LDS, then
// thread k < K adds the waves' sums in fixed order.  Result valid in threads k < K only
// (out_k).  `sh` holds (blockDim.x/64) * K doubles.  Deterministic.
template <int K>
__device__ __forceinline__ double block_sum_multi(const double (&v)[K], double* sh) {
    double w[K];
#pragma unroll
    for (int k = 0; k < K; ++k) w[k] = v[k];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
#pragma unroll
        for (int k = 0; k < K; ++k) w[k] += __shfl_xor(w[k], off, kWave);
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < K; ++k) sh[wv * K + k] = w[k];
    __syncthreads();
    double r = 0.0;
    if (threadIdx.x < K) {
        const int nw = blockDim.x / kWave;
        r = sh[threadIdx.x];
        for (int i = 1; i < nw; ++i) r += sh[i * K + threadIdx.x];
    }
    return r;
}

// ------------------------------------------------------------------ last-block hand-off
// Block-level partial record -> the block that arrives last reduces all records.
// Fence-free form of MI355X_MICROARCH.md "Valid forms", table row 1: every payload byte
// is stored write-through (`sc1`: relaxed agent-scope atomic stores) by the storing wave,
// which drains them (`s_waitcnt vmcnt(0)`) before ONE lane adds to the unsharded ticket;
// the block whose add returns nblocks-1 is last and reads every record with `sc1` loads
// (relaxed agent-scope atomic loads), so no release/acquire fence (~1.7 us each) is paid.
// The record's K values live in threads k < K of wave 0 (block_sum_multi's layout).
// `ticket` must be 0 at launch; the last block re-arms it to 0.
template <int K>
__device__ __forceinline__ bool publish_record_last(double* rec, double val, unsigned* ticket,
                                                    unsigned nblocks) {
    static_assert(K <= kWave, "record must be stored by wave 0");
    __shared__ int s_last;
    if (threadIdx.x < kWave) {  // wave 0 stores and signals
        if (threadIdx.x < K) __hip_atomic_store(rec + threadIdx.x, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (threadIdx.x == 0) {
            const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_last = (t == nblocks - 1);
            if (s_last) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    return s_last != 0;
}

// Fixed-order sum of `n` records of K doubles read with sc1 loads (see above); the sums
// end up in threads k < K (block_sum_multi layout).  `sh`: (blockDim.x/64) * K doubles.
// `nthr` (0 = blockDim.x): the threads that take records, so a block wider than the
// launch that normally runs this reduction sums them in the same order.
template <int K>
__device__ __forceinline__ double reduce_records(const double* recs, int n, double* sh, int nthr = 0) {
    double acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = 0.0;
    const int stride = nthr ? nthr : int(blockDim.x);
    #pragma unroll 1
    for (int i = int(threadIdx.x); i < n && int(threadIdx.x) < stride; i += stride)
#pragma unroll
        for (int k = 0; k < K; ++k)
            acc[k] += __hip_atomic_load(recs + int64_t(i) * K + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return block_sum_multi<K>(acc, sh);
}

// ------------------------------------------------------------------ 16-byte row vectors
// A logits row is split into [head | 16-B aligned body | tail]; head/tail have < EPV
// elements.  Traits per storage type:
struct F32T {
    static constexpr int kEPV = 4;        // elements per 16-B vector
    static constexpr uint32_t kNegInf = 0xff800000u;
    typedef float elem_t;
    __device__ static __forceinline__ float get(const vec4u& v, int e) {
        const uint32_t w = e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w;
        return __uint_as_float(w);
    }
    __device__ static __forceinline__ void unpack(const vec4u& v, float (&f)[kEPV]) {
        f[0] = __uint_as_float(v.x); f[1] = __uint_as_float(v.y);
        f[2] = __uint_as_float(v.z); f[3] = __uint_as_float(v.w);
    }
    __device__ static __forceinline__ vec4u pack(const float (&f)[kEPV]) {
        return vec4u_make(__float_as_uint(f[0]), __float_as_uint(f[1]),
                          __float_as_uint(f[2]), __float_as_uint(f[3]));
    }
    __device__ static __forceinline__ vec4u neg_inf() {
        return vec4u_make(kNegInf, kNegInf, kNegInf, kNegInf);
    }
    __device__ static __forceinline__ float load1(const void* row, int64_t j) {
        return reinterpret_cast<const float*>(row)[j];
    }
    __device__ static __forceinline__ void store1(void* row, int64_t j, float v) {
        reinterpret_cast<float*>(row)[j] = v;
    }
};
struct BF16T {
    static constexpr int kEPV = 8;
    static constexpr uint32_t kNegInf2 = 0xff80ff80u;
    typedef uint16_t elem_t;
    __device__ static __forceinline__ void unpack(const vec4u& v, float (&f)[kEPV]) {
        f[0] = bf_lo(v.x); f[1] = bf_hi(v.x); f[2] = bf_lo(v.y); f[3] = bf_hi(v.y);
        f[4] = bf_lo(v.z); f[5] = bf_hi(v.z); f[6] = bf_lo(v.w); f[7] = bf_hi(v.w);
    }
    __device__ static __forceinline__ vec4u pack(const float (&f)[kEPV]) {
        return vec4u_make(pack_bf2(f[0], f[1]), pack_bf2(f[2], f[3]),
                          pack_bf2(f[4], f[5]), pack_bf2(f[6], f[7]));
    }
    __device__ static __forceinline__ vec4u neg_inf() {
        return vec4u_make(kNegInf2, kNegInf2, kNegInf2, kNegInf2);
    }
    __device__ static __forceinline__ float load1(const void* row, int64_t j) {
        return bf2f(reinterpret_cast<const uint16_t*>(row)[j]);
    }
    __device__ static __forceinline__ void store1(void* row, int64_t j, float v) {
        reinterpret_cast<uint16_t*>(row)[j] = f2bf(v);
    }
};

// Geometry of one row: element pointer p (naturally aligned), V elements.
template <class DT>
struct RowSplit {
    int head;       // elements before the first 16-B boundary (< EPV)
    int64_t nvec;   // full 16-B vectors in the body
    int64_t tail0;  // first tail element
    int tail;       // tail elements (< EPV)
    __device__ __forceinline__ RowSplit(const void* p, int64_t V) {
        const uintptr_t a = reinterpret_cast<uintptr_t>(p);
        int h = int(((16u - (a & 15u)) & 15u) / sizeof(typename DT::elem_t));
        if (h > V) h = int(V);
        head = h;
        nvec = (V - h) / DT::kEPV;
        tail0 = h + nvec * DT::kEPV;
        tail = int(V - tail0);
    }
};

// 256-B line alignment of a row's vector grid.  A vector grid anchored at the row body's
// first 16-B boundary makes every 1-KB wave access straddle cache lines (a row of 50257
// bf16 starts at any 2-B phase), so each line is split between two instructions; shifting
// the lanes by line_shift(body) vectors makes every wave instruction cover whole 256-B
// spans (measured on MI355X, 512 x 13 x 16-B rows: 5.1 -> 5.8 TB/s read+write).  Vector i
// of the body is then handled by lane (i + shift) mod nthr at step (i + shift) / nthr.
constexpr int kLineVecs = 16;  // 16-B vectors per 256-B span; shift in [0, kLineVecs)
__device__ __forceinline__ int line_shift(const void* body) {
    return int((reinterpret_cast<uintptr_t>(body) >> 4) & (kLineVecs - 1));
}

// Opaque register copy: stops the compiler from keeping the unpacked fp32 copy of a
// register-resident bf16 row alive across the max / sum / store passes (it would double
// the row's VGPR footprint); unpacking again is 1-2 VALU ops per pair.
__device__ __forceinline__ void launder(vec4u& v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ int launder_int(int x) {
    asm volatile("" : "+v"(x));
    return x;
}

// Buffer resources (T8): a wave-uniform 128-bit descriptor in SGPRs + a 32-bit per-lane
// offset replaces a 64-bit address per 16-B vector (VGPR savings for register-resident
// rows), and the hardware range check turns out-of-row lanes into no-ops (loads read 0,
// stores are dropped).
constexpr int kRsrcFlags = 0x00020000;  // gfx950 raw buffer, dword3
constexpr int kAuxNT = 2;               // nt cache policy (streamed, read/written once)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, int(bytes), kRsrcFlags);
}

// Gradient-row store with a runtime cache policy (wave-uniform; trlx_set_tuning
// "store_policy"): kStoreNT = nt, kStoreSC1 = sc1 (MI355X_MICROARCH.md cache-policy bits:
// sc0 = 1, nt = 2, sc1 = 16).  nt measured best while a launch's gradient stream fits a few
// times in the 256 MB MALL (its dirty lines drain beside the next launch's reads); sc1 for
// multi-GB streams (C4 at 256-1024 rows: 2-5 % per step).
enum { kStoreNT = 0, kStoreNone = 1, kStoreSC1 = 2, kStoreSC0SC1 = 3, kStoreNTSC1 = 4 };
__device__ __forceinline__ void store_grad_b128(vec4u v, __amdgpu_buffer_rsrc_t r, int off, int spol) {
    switch (spol) {
        case kStoreNone: __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0); break;
        case kStoreSC1: __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16); break;
        case kStoreSC0SC1: __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 17); break;
        case kStoreNTSC1: __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 18); break;
        default: __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kAuxNT); break;
    }
}

// Streaming (read-once) 16-B load.
__device__ __forceinline__ vec4u ld_stream(const vec4u* p) {
    return __builtin_nontemporal_load(p);
}

}  // namespace trlx

// ------------------------------------------------------------------ host-side error plumbing
namespace trlx {
void set_error(const char* fmt, ...);
int check_launch(const char* what);
// A ragged batch's row order (vocab_rows.hip k_ragged_order): rows (b, t < lengths[b]) first in
// row order, then ~row of the padding rows, then the number of valid rows.  `order` holds
// ragged_order_bytes(B, T) bytes.
inline int64_t ragged_order_bytes(int64_t B, int64_t T) {  // list + count + the chunk counts of row_order.h
    return 4 * (B * T + 4 + (B * T + 1023) / 1024 + 1);
}
int launch_ragged_order(const int64_t* lengths, int64_t B, int64_t T, int* order, hipStream_t stream);

}  // namespace trlx

#define TRLX_REQUIRE(cond, code, ...)          \
    do {                                       \
        if (!(cond)) {                         \
            ::trlx::set_error(__VA_ARGS__);    \
            return (code);                     \
        }                                      \
    } while (0)
