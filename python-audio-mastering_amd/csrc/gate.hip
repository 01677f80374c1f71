// gate.hip — pyloudnorm's gated integrated loudness and the normalisation gain,
// on the device, so the chain runs without a host round trip (AME:212-222).
//
// pyloudnorm 0.1.1 Meter.integrated_loudness (mono, channel gain 1):
//   z_j   = (1/(0.4 rate)) * sum of K-weighted y^2 over block j (0.4 s, 0.1 s hop)
//   l_j   = -0.691 + 10 log10(z_j)
//   abs   : J_a = { j : l_j >= -70 }
//   rel   : Gamma_r = -0.691 + 10 log10(mean_{J_a} z) - 10
//   final : J_g = { j : l_j > Gamma_r and l_j > -70 },  L = -0.691 + 10 log10(mean_{J_g} z)
//           (nan_to_num: an empty J_g gives z = 0 -> L = -inf)
// AME:219-222: gain = 10 ** ((target - L) / 20).
// Block energies z_j: exactly pyloudnorm's (kw_blocks_kernel, numpy's float32
// reduction order) on the single-track and fused-batch chains; sums of 0.1 s
// segment energies (f64) on the time-sharded and per-stage paths (gate_blocks).
// The reductions over blocks are tree-ordered (the result differs from numpy's
// pairwise mean in the last bits only: ~1e-16 of the gain).
#include "common.h"

namespace mm {

struct GateArgs {
    int64_t n_blocks;
    const int32_t *blk_s0;  // first segment of block j
    const int32_t *blk_s1;  // one past its last segment
    const double *seg;      // segment energies
    double scale;           // 1 / (0.4 rate)
    double target;          // LUFS target
    double *out;            // [0] = L, [1] = gain
    const int64_t *trk_blk; // fused batch: block b gates track b's blocks [trk_blk[b], trk_blk[b+1])
                            // into out[2b], out[2b+1]; null: one track, blocks [0, n_blocks)
    double *zl;             // scratch [2 n_blocks]: z_j, then l_j (gate_blocks_kernel)
};

constexpr int GATE_THREADS = 1024;

// ---- exact block energies (pyloudnorm's z_j bit for bit) ----------------------
// pyloudnorm computes z_j = (1/(0.4 rate)) * np.sum(np.square(x[lo:hi])) with x the
// float32 K-weighted line: the squares are f32, np.sum is numpy's float32 add.reduce
// and the product with the Python float is f32 (NEP 50).  numpy reduces a contiguous
// array in buffer chunks of 8192 elements, res = 0 then res += pairwise(chunk), where
// pairwise(m) is: m < 8 a sequential sum; m <= 128 eight interleaved accumulators
// r[j] over elements j, j+8, ... combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), then
// the m % 8 tail in order; else pairwise(n2) + pairwise(m - n2), n2 = m/2 - (m/2)%8.
// The host turns that recursion into a program per distinct block length
// (mastering.hip pw_build, checked against np.sum on the CPU through mm_np_sum_f32):
//   ints [0..4]  nleaves, nnodes, nlevels, nchunks, root value (-1: empty sum)
//   then chunk_leaf[nchunks + 1], leaf_off[nleaves], leaf_len[nleaves],
//   node_a[nnodes], node_b[nnodes], level_node[nlevels + 1]
// values 0..nleaves-1 are the leaves, nleaves + k node k = val[a] + val[b]; nodes are
// sorted by height so each level only reads earlier ones.
struct KbArgs {
    const float *sq;          // tile-major f32 squares of the K-weighted line (kweight_kernel<true>)
    int64_t sq_stride;        // its row stride (tiles, a multiple of 4)
    int T;                    // frames per tile
    int64_t n_blocks;
    const int64_t *blk_lo;    // first frame of each block
    const int32_t *blk_prog;  // its program (int offset into prog)
    const int32_t *prog;
    float scale;              // f32(1 / (0.4 rate))
    double *zl;               // [2 n_blocks]: z_j, then l_j (read by gate_kernel)
};
constexpr int KB_CHUNK = 8192;   // numpy's reduction buffer (elements)
constexpr int KB_VMAX = 2048;    // leaves + nodes of one block (76 800 frames at 192 kHz: ~1200)
constexpr int KB_THREADS = 256;
constexpr int KB_LD = 13;        // 16-byte loads per thread per chunk: rows T <= 512 x (8192/T + 8)/4 tile quads
__host__ __device__ constexpr int kb_pad(int i) { return i + 4 * (i >> 7); }  // 128-element runs 4 banks apart

// One workgroup per block; consecutive blocks on one XCD (their windows overlap
// 3/4: the re-reads hit that XCD's L2).  Per 8192-element chunk: the chunk's
// frames are staged in LDS (16-byte loads of 4 tiles at a row, the next chunk's
// loads in flight while this one is summed), four lanes per leaf run numpy's eight
// accumulators (two each), then the program's levels combine the leaves in numpy's
// order.
__global__ void __launch_bounds__(KB_THREADS) kw_blocks_kernel(KbArgs a) {
    __shared__ __attribute__((aligned(16))) float el[kb_pad(KB_CHUNK)];
    __shared__ float val[KB_VMAX];
    const unsigned per = gridDim.x / 8;  // (the grid is a multiple of 8)
    const int64_t j = (int64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
    if (j >= a.n_blocks) return;  // (workgroup-uniform)
    const int tid = threadIdx.x;
    const int32_t *P = a.prog + a.blk_prog[j];
    const int nl = P[0], nn = P[1], nlev = P[2], nch = P[3], root = P[4];
    const int32_t *chunk_leaf = P + 5, *loff = chunk_leaf + nch + 1, *llen = loff + nl, *na = llen + nl,
                  *nb = na + nn, *lvl = nb + nn;
    const int64_t lo = a.blk_lo[j];
    const int T = a.T;
    const float4 *sq4 = reinterpret_cast<const float4 *>(a.sq);
    const int64_t rs4 = a.sq_stride / 4;
    float4 buf[KB_LD];
    int64_t gq0 = 0;   // the staged chunk's first tile quad
    int nq = 0;        // its tile quads per row
    auto issue = [&](int c) __attribute__((always_inline)) {  // chunk c's loads into buf
        const int64_t F0 = lo + (int64_t)c * KB_CHUNK;
        const int m = loff[chunk_leaf[c + 1] - 1] + llen[chunk_leaf[c + 1] - 1] - c * KB_CHUNK;
        gq0 = (F0 / T) >> 2;
        nq = (int)(((F0 + m - 1) / T >> 2) - gq0 + 1);
#pragma unroll
        for (int r = 0; r < KB_LD; ++r) {
            const int k = tid + r * KB_THREADS;
            const int n = k / nq, q = k - n * nq;
            buf[r] = n < T ? sq4[(int64_t)n * rs4 + gq0 + q] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    if (nch > 0) issue(0);
    for (int c = 0; c < nch; ++c) {
        const int l0 = chunk_leaf[c], l1 = chunk_leaf[c + 1];
        const int64_t F0 = lo + (int64_t)c * KB_CHUNK;
        const int m = loff[l1 - 1] + llen[l1 - 1] - c * KB_CHUNK;  // the chunk's length
#pragma unroll
        for (int r = 0; r < KB_LD; ++r) {
            const int k = tid + r * KB_THREADS;
            const int n = k / nq, q = k - n * nq;
            const int64_t i0 = ((gq0 + q) * 4) * T + n - F0;  // chunk index of tile 4(gq0+q), row n
            const float e4[4] = {buf[r].x, buf[r].y, buf[r].z, buf[r].w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int64_t i = i0 + (int64_t)e * T;
                if (n < T && i >= 0 && i < m) el[kb_pad((int)i)] = e4[e];
            }
        }
        __syncthreads();
        if (c + 1 < nch) issue(c + 1);  // in flight while this chunk is summed
        const int q = tid & 3;          // accumulators 2q, 2q + 1 of the leaf
        for (int li = l0 + (tid >> 2); li < l1; li += KB_THREADS / 4) {
            const int off = loff[li] - c * KB_CHUNK, len = llen[li];
            float res;
            if (len < 8) {  // (a chunk shorter than 8: numpy's sequential sum; lane 0 of the four)
                res = el[kb_pad(off)];
                for (int i = 1; i < len; ++i) res = __fadd_rn(res, el[kb_pad(off + i)]);
            } else {
                float2 r = *reinterpret_cast<const float2 *>(el + kb_pad(off) + 2 * q);
                const int full = len - (len & 7);
                int i = 8;
                for (; i < full; i += 8) {
                    const float2 v = *reinterpret_cast<const float2 *>(el + kb_pad(off + i) + 2 * q);
                    r.x = __fadd_rn(r.x, v.x);
                    r.y = __fadd_rn(r.y, v.y);
                }
                // ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)); f32 addition commutes, so every lane
                // of the four ends with the same bits
                float p = __fadd_rn(r.x, r.y);
                p = __fadd_rn(p, __shfl_xor(p, 1));
                res = __fadd_rn(p, __shfl_xor(p, 2));
                for (; i < len; ++i) res = __fadd_rn(res, el[kb_pad(off + i)]);
            }
            if (q == 0) val[li] = res;
        }
        __syncthreads();  // (the next chunk overwrites el)
    }
    for (int L = 0; L < nlev; ++L) {
        for (int k = lvl[L] + tid; k < lvl[L + 1]; k += KB_THREADS) val[nl + k] = __fadd_rn(val[na[k]], val[nb[k]]);
        __syncthreads();
    }
    if (tid == 0) {
        const float s = root < 0 ? 0.0f : val[root];
        const double z = (double)__fmul_rn(a.scale, s);
        a.zl[j] = z;
        a.zl[a.n_blocks + j] = -0.691 + 10.0 * log10(z);
    }
}

// z_j and l_j of every block, one thread per block (the segment sum in segment
// order, as the host restatement): the gate itself then streams them coalesced.
// (Round 5 computed them inside the one-workgroup gate, a dependent chain of
// segment loads per block and thread: 220 us for a 2-hour track, 13 us for C2.)
constexpr int GATE_BLK_THREADS = 256;
__global__ void __launch_bounds__(GATE_BLK_THREADS) gate_blocks_kernel(GateArgs a) {
    const int64_t j = (int64_t)blockIdx.x * GATE_BLK_THREADS + threadIdx.x;
    if (j >= a.n_blocks) return;
    const int32_t s0 = a.blk_s0[j], s1 = a.blk_s1[j];
    double acc = 0.0;
    for (int32_t s = s0; s < s1; ++s) acc += a.seg[s];
    const double z = a.scale * acc;
    a.zl[j] = z;
    a.zl[a.n_blocks + j] = -0.691 + 10.0 * log10(z);
}

// sum and count over the block, result broadcast to every thread: a fixed-order
// butterfly within each wave, then the waves' partials in order (deterministic)
__device__ __forceinline__ void gate_reduce(double &sum, long long &cnt, double *rs, long long *rc) {
    const int t = threadIdx.x;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        sum += __shfl_xor(sum, o);
        cnt += __shfl_xor(cnt, o);
    }
    if ((t & 63) == 0) {
        rs[t >> 6] = sum;
        rc[t >> 6] = cnt;
    }
    __syncthreads();
    sum = 0.0;
    cnt = 0;
#pragma unroll
    for (int w = 0; w < GATE_THREADS / 64; ++w) {
        sum += rs[w];
        cnt += rc[w];
    }
    __syncthreads();
}

// One workgroup per track over its blocks' (z, l) from gate_blocks_kernel: thread t
// sums blocks t, t + 1024, ... in order, then the fixed-order reduction.
__global__ void __launch_bounds__(GATE_THREADS) gate_kernel(GateArgs a) {
    __shared__ double rs[GATE_THREADS / 64];
    __shared__ long long rc[GATE_THREADS / 64];
    const int t = threadIdx.x;
    const int64_t j0 = a.trk_blk ? a.trk_blk[blockIdx.x] : 0;
    const int64_t j1 = a.trk_blk ? a.trk_blk[blockIdx.x + 1] : a.n_blocks;
    double *out = a.out + 2 * blockIdx.x;
    const double *zv = a.zl, *lv = a.zl + a.n_blocks;
    double sum = 0.0;
    long long cnt = 0;
#pragma unroll 8
    for (int64_t j = j0 + t; j < j1; j += GATE_THREADS) {
        const double z = zv[j], l = lv[j];
        if (l >= -70.0) {
            sum += z;
            ++cnt;
        }
    }
    gate_reduce(sum, cnt, rs, rc);
    const double mean_abs = cnt ? sum / (double)cnt : __longlong_as_double(0x7ff8000000000000LL);
    const double gamma_r = -0.691 + 10.0 * log10(mean_abs) - 10.0;
    sum = 0.0;
    cnt = 0;
#pragma unroll 8
    for (int64_t j = j0 + t; j < j1; j += GATE_THREADS) {
        const double z = zv[j], l = lv[j];
        if (l > gamma_r && l > -70.0) {
            sum += z;
            ++cnt;
        }
    }
    gate_reduce(sum, cnt, rs, rc);
    if (t == 0) {
        const double zavg = cnt ? sum / (double)cnt : 0.0;
        const double L = -0.691 + 10.0 * log10(zavg);
        out[0] = L;
        out[1] = pow(10.0, (a.target - L) / 20.0);
    }
}

}  // namespace mm
