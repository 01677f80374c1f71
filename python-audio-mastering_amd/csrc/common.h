// common.h — shared device-side argument blocks of the mastering kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Python float / numpy semantics: no implicit FMA contraction anywhere.  The
// linear-recurrence kernels call fma() explicitly where it is wanted.
#pragma clang fp contract(off)

namespace mm {

// Software-pipelined sequential stream: ld() yields the next element (called in
// order), proc(v) consumes elements in order.  NB*B elements stay in flight in
// registers, hiding HBM/Infinity-Cache latency behind a lane's dependent chain.
template <int B, int NB, typename V, typename LD, typename PROC>
__device__ __forceinline__ void stream(int len, LD &&ld, PROC &&proc) {
    V buf[NB][B];
#pragma unroll
    for (int k = 0; k < NB; ++k)
#pragma unroll
        for (int j = 0; j < B; ++j)
            if (k * B + j < len) buf[k][j] = ld();
    for (int n0 = 0; n0 < len; n0 += NB * B) {
#pragma unroll
        for (int k = 0; k < NB; ++k) {
#pragma unroll
            for (int j = 0; j < B; ++j)
                if (n0 + k * B + j < len) proc(buf[k][j]);
#pragma unroll
            for (int j = 0; j < B; ++j)
                if (n0 + (k + NB) * B + j < len) buf[k][j] = ld();
        }
    }
}

struct SatArgs {
    float keep, mix, drive;
    int on;
};

// Arguments of the pre-chain (EQ) and crossover kernels.
struct StageArgs {
    const float *in;   // natural interleaved f32 input (stage A)
    int64_t N_in;      // valid input frames
    int64_t N_proc;    // processed timeline frames
    int64_t G;         // tiles
    int T;             // frames per tile
    int ch;            // channels (1|2)
    SatArgs sat;
    double width;
    int width_on;
    double sos[4][5];  // {b0,b1,b2,a1,a2}
    double *z_out;     // pass 1: per-tile zero-state end state [G][ch][D]
    const double *s_in;  // pass 2: per-tile carry-in state [G][ch][D]
    const short2 *q_in;  // tile-major int16 pairs
    short2 *q_out;
    short2 *band_out[3];
};

struct CompArgs {
    int64_t N_proc, G;
    int T, K, ch, warmup;
    int S;                     // tiles per super-tile (envelope solve unit)
    int64_t GS;                // super-tiles (chunks * ceil(K/S))
    const short2 *band[3];
    const double *max_att[3];  // device LUTs [32769]
    int look[3];
    double attack_frames[3], release_frames[3];
    double rcp_attack[3], rcp_release[3];
    double *M[3];              // tile-major per-frame max attenuation
    double *start[3];          // per-super-tile speculative start state
    double *tstart[3];         // per-tile start state (recorded by the walks)
    const double *end_in[3];
    double *end_out[3];
    unsigned int *changed;
    int32_t *ident[3];         // per super-tile: 1 if every frame has M == 0 (identity map)
    int32_t *prev_active[3];   // per super-tile: nearest earlier non-identity one in the chunk, -1 if none
    short2 *q_out;
};

struct KwArgs {
    int64_t N_proc, G;
    int T, ch;
    double sos[2][5];
    const short2 *mix;
    double *z_out;
    const double *s_in;
    int64_t n_segs;
    const int64_t *seg_bounds;
    double *part;      // [G][2]
    int64_t *part_seg; // [G]
};

struct FinArgs {
    int64_t N_proc, G;
    int T, ch, out_kind, use_gain;
    double gain;
    const short2 *mix;
    void *out;
};

// Affine state scan over tiles of independent lines (chunks x channels).
struct ScanArgs {
    int dim;            // state dim per channel (<= 8)
    int c;              // tiles per thread
    int ch;             // channels interleaved in z: [tile][ch][dim]
    int64_t line_tiles; // tiles per line (last line may be shorter)
    int64_t G;          // total tiles
    const double *phi;      // [8*8]  one tile
    const double *phi_pow;  // [MM_SCAN_POWERS][8*8]  Phi^(c*2^k)
    const double *phi_last; // [8*8]  last tile of a line
    const double *z;        // per-tile zero-state end state
    double *s;              // per-tile carry-in state (exclusive prefix)
    const double *init;     // optional per-line initial state [lines][ch][dim] (or null)
    double *line_end;       // optional per-line end state [lines][ch][dim] (or null)
};

}  // namespace mm
