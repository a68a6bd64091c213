// Valid-rows-first orders of a batch's rows, two launches over 1024-row chunks: per-chunk valid
// counts, then every chunk sums the counts before it (O(N/1024) loads per workgroup, no pass
// over the batch by one workgroup) and places its rows.  order[0, nv) = the valid rows in row
// order, order[nv, N) = ~row of the others in row order, order[N] = nv.
//   mask form (LEN = false): row p is valid iff mask[p] != 0 (the fused loss side's compaction)
//   lengths form (LEN = true): row p = b·T + j is valid iff j < clamp(lengths[b], 0, T) (a ragged
//   batch's decoder lengths, vocab_rows.hip / lmhead_rows.hip)
#pragma once
#include "common.h"

namespace trlx {

constexpr int kOrderChunk = 1024;  // rows per workgroup of the two order launches (256 threads x 4)

template <bool LEN>
__device__ __forceinline__ bool order_valid(const int64_t* src, int T, int64_t p) {
    if (LEN) {
        const int64_t b = p / T;
        return p - b * T < src[b];  // j < lengths[b] (a negative length: no valid row)
    }
    return src[p] != 0;
}

template <bool LEN>
__global__ __launch_bounds__(256) void k_order_count(const int64_t* src, int T, int64_t n, int* cnt) {
    __shared__ int s_red[4];
    const int64_t p0 = int64_t(blockIdx.x) * kOrderChunk;
    int c = 0;
    for (int64_t p = p0 + threadIdx.x; p < min(p0 + kOrderChunk, n); p += blockDim.x) c += order_valid<LEN>(src, T, p);
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) cnt[blockIdx.x] = s_red[0] + s_red[1] + s_red[2] + s_red[3];
}

template <bool LEN>
__global__ __launch_bounds__(256) void k_order_place(const int64_t* src, int T, int64_t n, const int* cnt, int nchunk,
                                                     int* order) {
    __shared__ int s_red[2][4];
    __shared__ int s_wsum[4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    int pre = 0, tot = 0;
    for (int c = tid; c < nchunk; c += blockDim.x) {
        tot += cnt[c];
        pre += c < int(blockIdx.x) ? cnt[c] : 0;
    }
    for (int off = 32; off > 0; off >>= 1) {
        tot += __shfl_xor(tot, off);
        pre += __shfl_xor(pre, off);
    }
    const int64_t p0 = int64_t(blockIdx.x) * kOrderChunk + 4 * tid;  // 4 consecutive rows per thread
    int f[4], loc = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        f[e] = p0 + e < n && order_valid<LEN>(src, T, p0 + e);
        loc += f[e];
    }
    int inc = loc;  // inclusive scan of the threads' counts within the wave
    for (int off = 1; off < 64; off <<= 1) {
        const int u = __shfl_up(inc, off);
        inc += lane >= off ? u : 0;
    }
    if (lane == 0) {
        s_red[0][w] = tot;
        s_red[1][w] = pre;
    }
    if (lane == 63) s_wsum[w] = inc;
    __syncthreads();
    const int nvalid = s_red[0][0] + s_red[0][1] + s_red[0][2] + s_red[0][3];
    int run = s_red[1][0] + s_red[1][1] + s_red[1][2] + s_red[1][3];
    for (int k = 0; k < w; ++k) run += s_wsum[k];
    run += inc - loc;  // valid rows before p0
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int64_t p = p0 + e;
        if (p >= n) break;
        if (f[e])
            order[run++] = int(p);
        else
            order[nvalid + int(p - run)] = ~int(p);
    }
    if (blockIdx.x == 0 && tid == 0) order[n] = nvalid;
}

// Scratch ints of the two launches' chunk counts for n rows.
inline int64_t order_chunks(int64_t n) { return (n + kOrderChunk - 1) / kOrderChunk; }

template <bool LEN>
inline int launch_order(const int64_t* src, int T, int64_t n, int* cnt, int* order, hipStream_t s) {
    const unsigned nchunk = unsigned(order_chunks(n));
    hipLaunchKernelGGL(k_order_count<LEN>, dim3(nchunk), dim3(256), 0, s, src, T, n, cnt);
    int rc = check_launch("k_order_count");
    if (rc) return rc;
    hipLaunchKernelGGL(k_order_place<LEN>, dim3(nchunk), dim3(256), 0, s, src, T, n, cnt, int(nchunk), order);
    return check_launch("k_order_place");
}

}  // namespace trlx
