// Deep-stack C=16 path (BASELINE config C3, antisym-ResNet-110: 108 Euler
// blocks at 32x32x16): LDS temporal fusion.  One 32x32x16 bf16 image is
// 32 KiB, so a workgroup keeps the whole image resident in LDS and runs ALL
// L Euler steps on it, instead of one HBM round trip per block:
//
//   x_{l+1} = x_l + h * relu(conv3x3(x_l, W_l) + b_l)      l = 0 .. L-1
//
// (single_layer_identity_block, models/tfkeras_resnets.py:69-92, with the
// antisymmetric kernel of layers/tfkeras_layer_Conv2DAntisymmetric3By3.py
// :157-171 materialised by asr_theta_to_w).  Training stores every x_{l+1}
// (the backward's weight gradient reads it) and the relu mask; inference
// stores only x_L.  HBM traffic per block: one activation write (+ the 1/16
// mask) instead of a read and a write.
//
// Conv = implicit GEMM on v_mfma_f32_16x16x32_bf16 over kappa = (tap, i):
//   Z^T[o][p] = b[o] + sum_kappa W^T[o][kappa] X[p][kappa]
// with the 9 taps paired into 5 k-steps so that B fragments are shared
// between output rows ("row-reuse" order):
//   ks 0..2: taps (ky, 0) | (ky, 1) of tile row r + ky   -> fragment F(r + ky)
//   ks 3:    taps (0, 2)  | (1, 2)  of tile rows r, r+1  -> fragment G(r)
//   ks 4:    taps (2, 2)  | zero    of tile rows r+2, r+3 -> fragment G(r + 2)
// F(R) serves output rows R-2 .. R and G(R) rows R and R-2, so a wave reads
// each of its 10 tile rows twice (F, G) instead of 10 fragments per output
// row.  A = W^T (5 k-steps, the pad half multiplies the zero tap 9 of the
// standard packing) in VGPRs per layer, gathered from asr_theta_to_w's
// packing by a per-lane permutation.
//
// LDS tile: 34 x 34 pixels (zero halo) x 32 B; chunk c (channels 8c..8c+7)
// of tile column tc is stored at tc*32 + 16*(c ^ bit2(tc)).  The swizzle
// makes the 16-B epilogue stores (ds_write_b128: 8 lanes, banks mod 32)
// conflict-free and keeps the B reads (ds_read_b128 lane groups, banks mod
// 64) conflict-free.  The accumulators of a row's two pixel tiles are
// regrouped with v_permlane16_swap so each lane owns 8 consecutive channels
// of one pixel: one 16-B LDS store, one 16-B global store and one mask byte
// per lane and row, and the residual x stays in the lane's registers.
#include <type_traits>

#include "asr_common.h"
#include "asr_device.h"

namespace asr {
namespace deep {

using namespace blk;

#ifndef ASR_DEEP_TRACE
#define ASR_DEEP_TRACE 0  // diagnostic build only: per-step s_memtime stamps of workgroup 0 (tools/tracebench.py)
#endif

constexpr int C = 16, W = 32, H = 32, TW = W + 2;
constexpr int ROWB = TW * C * 2;       // 1088 B per tile row (halo columns included)
constexpr int TILE = (H + 2) * ROWB;   // 36992 B per image tile (halo rows included)
constexpr int IMG = H * W * C;         // elements per image
constexpr int KS = 5;                  // k-steps of 32 over kappa = 9 taps x 16 channels (+ zero tap)
constexpr int WSTRIDE = KS * 512;      // packed W^T elements per layer (asr_wpack_elems(16))
constexpr int NWAVE = 4;               // forward waves per workgroup; wave w owns image rows [8w, 8w+8)
constexpr int RPW = H / NWAVE;
constexpr int ROW_G = W * C * 2;       // 1024 B per image row in HBM

static __device__ float g_zero_bias[C];  // bias of layers without one (never written)

typedef unsigned u32x4v __attribute__((ext_vector_type(4)));

// byte offset of chunk c of tile column tc within a tile row
__device__ __forceinline__ unsigned swz(int tc, int c) { return (unsigned)(tc * 32 + 16 * (c ^ ((tc >> 2) & 1))); }

// per-lane element offsets of the 5 A fragments within one layer's packed
// W^T: lane (o, kg) of row-reuse k-step ks needs tap t (first of the pair for
// kg < 2), channels 8(kg&1)..+7, found in the standard packing at k-step
// t/2, lane group 2(t&1) + (kg&1)
__device__ __forceinline__ void wt_offsets(int lane, unsigned (&wo)[KS]) {
  const int o = lane & 15, kg = lane >> 4, sec = kg >> 1;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int t = ks < 3 ? 3 * ks + sec : (ks == 3 ? 2 + 3 * sec : 8 + sec);
    wo[ks] = (unsigned)(((t >> 1) * 64 + o + 16 * ((t & 1) * 2 + (kg & 1))) * 8);
  }
}
__device__ __forceinline__ void load_wt(const bf16* __restrict__ w, const unsigned (&wo)[KS], bf16x8 (&A)[KS]) {
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) A[ks] = *(const bf16x8*)(w + wo[ks]);
}

using blk::bit01;
using blk::f32x2;
using blk::hi_f;
using blk::lo_f;
using blk::lshl_or;
using blk::pk_bf16;
using blk::pk_fma;
using blk::regroup;
using blk::static_for;

// One output row of the implicit GEMM for both pixel tiles from the row-reuse
// fragments (fixed accumulation order: init, k-steps 0..4).
__device__ __forceinline__ void row_mfma(const bf16x8 (&A)[KS], const bf16x8 (&F0)[2], const bf16x8 (&F1)[2],
                                         const bf16x8 (&F2)[2], const bf16x8 (&G0)[2], const bf16x8 (&G2)[2],
                                         f32x4 (&acc)[2]) {
#pragma unroll
  for (int pt = 0; pt < 2; ++pt) acc[pt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], F0[pt], acc[pt], 0, 0, 0);
#pragma unroll
  for (int pt = 0; pt < 2; ++pt) acc[pt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1], F1[pt], acc[pt], 0, 0, 0);
#pragma unroll
  for (int pt = 0; pt < 2; ++pt) acc[pt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[2], F2[pt], acc[pt], 0, 0, 0);
#pragma unroll
  for (int pt = 0; pt < 2; ++pt) acc[pt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[3], G0[pt], acc[pt], 0, 0, 0);
#pragma unroll
  for (int pt = 0; pt < 2; ++pt) acc[pt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[4], G2[pt], acc[pt], 0, 0, 0);
}

// Row-reuse B fragments of the wave's 10 tile rows: F(R), G(R) for R = j..j+3
// live in a ring of 4 (slot R & 3); row j's MFMAs read F(j..j+2), G(j), G(j+2)
// while the fragments of tile row j+3 load.
// (NS = 3: tile row j+3 loads into row j's slots after row j's MFMAs issue)
template <int NS = 4>
struct FragT {
  bf16x8 F[NS][2], G[NS][2];
  __device__ __forceinline__ void load(const unsigned char* tile, unsigned bF, unsigned bG, int R) {
#pragma unroll
    for (int pt = 0; pt < 2; ++pt) {
      F[R % NS][pt] = *(const bf16x8*)(tile + bF + R * ROWB + pt * 512);
      G[R % NS][pt] = *(const bf16x8*)(tile + bG + R * ROWB + pt * 512);
    }
  }
};
using Frag = FragT<4>;

// x_{l+1} for l = 0 .. L-1 of every image the workgroup owns.
//   x0:    [N,32,32,16] bf16 (the stem output)
//   y0:    output of layer 0; layer l writes y0 + l*y_stride (STORE_ALL), or
//          only layer L-1 writes y0 (inference)
//   mask0: relu masks (MASK), layer l at mask0 + l*mask_stride bytes; per
//          pixel 16 bits, bit c = channel c
//   wpack: packed W^T, layer l at wpack + l*WSTRIDE; bias: layer l at bias + l*bias_stride
template <bool STORE_ALL, bool MASK>
__global__ __launch_bounds__(64 * NWAVE, 2) void k_fwd16_fused(const bf16* __restrict__ x0, bf16* __restrict__ y0,
                                                            long y_stride, uint8_t* __restrict__ mask0,
                                                            long mask_stride, const bf16* __restrict__ wpack,
                                                            const float* __restrict__ bias, long bias_stride,
                                                            float h, int N, int L) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, lx = lane & 15;
  const int r0 = wave * RPW;
  // both tiles and the zero row behind them (G(33) of the second tile reads it)
  for (int i = tid; i < (2 * TILE + ROWB) / 16; i += 64 * NWAVE) ((uint4*)lds)[i] = make_uint4(0, 0, 0, 0);
  const unsigned bF = (unsigned)(r0 * ROWB) + swz(lx + (g >> 1), g & 1);
  const unsigned bG = (unsigned)((r0 + (g >> 1)) * ROWB) + swz(lx + 2, g & 1);
  const int px = lx + 16 * (g & 1), cg = g >> 1;  // the lane's pixel / channel chunk after regroup
  const unsigned oT = (unsigned)((r0 + 1) * ROWB) + swz(px + 1, cg);
  const unsigned oG = (unsigned)(((r0 * W + px) * C + 8 * cg) * 2);
  const unsigned oM = (unsigned)((r0 * W + px) * 2 + cg);
  unsigned wo[KS];
  wt_offsets(lane, wo);
  // branch-free prefetch below (loads on a conditional path make the compiler's
  // loop-header wait vmcnt(0), which would also wait for the previous layer's stores)
  const float* bsrc = bias ? bias : g_zero_bias;
  const long bstr = bias ? bias_stride : 0;
  __syncthreads();

  for (int n = blockIdx.x; n < N; n += gridDim.x) {
    // x0 of image n: the lane's own chunks (the residual of layer 0) into tile 0
    const unsigned char* xin = (const unsigned char*)(x0 + (long)n * IMG);
    bf16x8 xr[RPW];
#pragma unroll
    for (int j = 0; j < RPW; ++j) xr[j] = *(const bf16x8*)(xin + oG + j * ROW_G);
#pragma unroll
    for (int j = 0; j < RPW; ++j) *(bf16x8*)(lds + oT + j * ROWB) = xr[j];
    bf16x8 A[KS], An[KS];
    load_wt(wpack, wo, A);
    float bz[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) bz[e] = bsrc[4 * g + e];
    barrier_lds();

    for (int l = 0; l < L; ++l) {
      const unsigned char* src = lds + (l & 1) * TILE;
      unsigned char* dst = lds + ((l + 1) & 1) * TILE;
      const int ln = min(l + 1, L - 1);
      float bn[4];
      // next layer's W^T fragments and bias (L2-resident) while this one runs
      // (copied to A / bz at the layer end: alternating two register sets
      // instead makes this kernel spill)
      load_wt(wpack + (long)ln * WSTRIDE, wo, An);
#pragma unroll
      for (int e = 0; e < 4; ++e) bn[e] = bsrc[ln * bstr + 4 * g + e];
      const bool store = STORE_ALL || l == L - 1;
      unsigned char* yl = (unsigned char*)(y0 + (STORE_ALL ? (long)l * y_stride : 0) + (long)n * IMG);
      uint8_t* ml = MASK ? mask0 + (long)l * mask_stride + (long)n * (IMG / 8) : nullptr;
      Frag fr;
#pragma unroll
      for (int R = 0; R < 3; ++R) fr.load(src, bF, bG, R);
#pragma unroll
      for (int j = 0; j < RPW; ++j) {
        if (j + 3 <= RPW + 1) fr.load(src, bF, bG, j + 3);
        f32x4 acc[2] = {{bz[0], bz[1], bz[2], bz[3]}, {bz[0], bz[1], bz[2], bz[3]}};
        row_mfma(A, fr.F[j & 3], fr.F[(j + 1) & 3], fr.F[(j + 2) & 3], fr.G[j & 3], fr.G[(j + 2) & 3], acc);
        // epilogue on the regrouped chunk: y = x + h * relu(z) (fp32, one rounding),
        // relu bits as TF's ReluGrad (z > 0)
        float z[8];
        regroup(acc[0], acc[1], z);
        const u32x4v xw = __builtin_bit_cast(u32x4v, xr[j]);
        u32x4v yw;
        unsigned bits = 0;
        static_for<0, 4>([&](auto dc) {
          constexpr int d = decltype(dc)::value;
          // relu on the bit pattern: a float is > 0 iff its bits are a positive int
          const int ra = max(__float_as_int(z[2 * d]), 0), rb = max(__float_as_int(z[2 * d + 1]), 0);
          yw[d] = pk_bf16(fmaf(h, __int_as_float(ra), lo_f(xw[d])), fmaf(h, __int_as_float(rb), hi_f(xw[d])));
          bits = d == 0 ? bit01(ra) : lshl_or<2 * d>(bit01(ra), bits);
          bits = lshl_or<2 * d + 1>(bit01(rb), bits);
        });
        const bf16x8 y = __builtin_bit_cast(bf16x8, yw);
        *(bf16x8*)(dst + oT + j * ROWB) = y;
        // streaming (nt) stores: x_{l+1} and its mask are read back only by the backward
        // (+6 % forward, -1 % backward against default-policy stores, A/B r02k)
        if (store) __builtin_nontemporal_store(yw, (u32x4v*)(yl + oG + j * ROW_G));
        if (MASK) __builtin_nontemporal_store((uint8_t)bits, ml + oM + j * 64);
        xr[j] = y;
      }
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) A[ks] = An[ks];
#pragma unroll
      for (int e = 0; e < 4; ++e) bz[e] = bn[e];
      barrier_lds();  // layer l+1's tile complete; layer l's tile free
    }
  }
}


// ---------------------------------------------------------------------------
// Backward, fused over the stack.  Per image, layers L-1 .. 0:
//   dzm  = dx_{l+1} & mask_l                       (dz = h*dzm; bf16 bit mask)
//   dx_l = dx_{l+1} - h*conv(dzm, W_l) + 2*gamma*h*dzm   (A^T = -A + 2 gamma I;
//          for non-antisymmetric kinds W_l is W_bwd = -flip(W)^T, gamma 0)
//   dW_l += h * sum_p x_l[p + s(tap)] (x) dzm[p],  db_l += h * sum_p dzm[p]
// The layers run in segments of KSEG: the weight gradients of a segment's
// layers accumulate in registers over all images of the workgroup, so each
// layer gets ONE slab [dW (9*16*16) | db (16)] fp32 per workgroup (the layout
// asr_api's reduce_slabs_to_groups / project_layers consume), and dx crosses
// HBM only at segment boundaries.
//
// One 512-thread workgroup per CU, two waves per SIMD with split roles:
//   waves 0-3 (dgrad): image rows [8w, 8w+8): the forward's row-reuse implicit
//     GEMM on the dzm tile; dx of the wave's pixels stays in registers (the
//     regrouped layout), and the epilogue writes dzm_{l-1} = dx_l & mask_{l-1}
//     straight into the other dz tile (no separate masking pass), plus db;
//   waves 4-6 (wgrad): tap column kx = w-4 of all 32 rows: a GEMM with M = the
//     tap's 16 input channels, N = o, K = the 32 pixels of a row.  The x
//     fragment of image row i (ds_read_b64_tr_b16, T10) serves the three taps
//     (ky, kx) of output rows i+1-ky, so every x row is read once per wave;
//     the dz fragments of the last three rows stay in registers.  The 8
//     k-pixels of lane group g are 8g + 4*(hh ^ (g & 1)) + q for the two reads
//     hh: odd groups swap halves, so the lane groups read disjoint banks;
//   wave 7 DMAs x_{l-1} and mask_{l-2} (the dgrad epilogue of layer l-1 needs
//     mask_{l-2}) meanwhile, and at an image's last layer the next image's
//     x_ltop and masks; the dgrad waves load the next image's dx then.
// One barrier per layer.  LDS: 2 dz tiles (swizzled, zero halo) + zero row |
// 2 x tiles (image rows, zero halo columns) | 2 x 2 KiB masks | db partials.
// ---------------------------------------------------------------------------
constexpr int WDEPTH = 2;   // wgrad waves: x / dz row fragments read this many rows ahead of their MFMAs (3: flat, r04p)
constexpr int NDG = 8;      // dgrad waves (image rows split among them; 4 waves: slower, r02i)
constexpr int RPB = H / NDG;  // image rows per dgrad wave
constexpr int KSEG = 8;     // layers per segment (dW accumulators in registers)
constexpr int NWB = NDG + 4;             // waves per backward workgroup: dgrad, 3 wgrad, staging
constexpr int ES = 9 * C * C + C;        // slab floats per layer
constexpr int XT = H * ROWB;             // x tile: 32 image rows x 34 columns
constexpr int MB = IMG / 8;              // 2 KiB of relu bits per image
// x tile rows [0, XS) reach LDS through wave 7's registers (loaded two steps
// ahead, written one step ahead); rows [XS, 32) by LDS-DMA two steps ahead into
// a rotation of three row blocks: the upper rows of the two x tiles and L_E.
constexpr int XS = 22;
constexpr int L_Z = 0, L_X = L_Z + 2 * TILE + ROWB, L_M = L_X + 2 * XT, L_TAB = L_M + 2 * MB;
constexpr int L_DB = L_TAB + 16 * 8;   // after the mask nibble -> 4 x 0xffff/0 bf16 AND-mask table
constexpr int L_E = L_DB + KSEG * C * 4;  // after the segment's db sums [KSEG][C]
constexpr int L_TOTAL = L_E + (H - XS) * ROWB;
__device__ __forceinline__ int xhi_base(int t) {  // LDS offset of image row XS of step t's x
  const int r = t % 3;
  return r == 2 ? L_E : L_X + r * XT + XS * ROWB;
}
static_assert(L_TOTAL <= 160 * 1024, "LDS budget");

__device__ __forceinline__ bf16x8 tr2(const unsigned char* base, const unsigned (&o)[2]) {
  return tr_pair(base + o[0], base + o[1]);
}

// 8 bf16 ANDed with the relu bits of the lane's mask byte (table per nibble:
// 0xffff per set bit; 16 entries of 8 B, so lanes of a read group share
// entries by broadcast and never conflict)
__device__ __forceinline__ u32x4v mask_bf16x8(const unsigned char* lds, u32x4v v, unsigned m) {
  const u32x2 lo = *(const u32x2*)(lds + L_TAB + (m & 15u) * 8), hi = *(const u32x2*)(lds + L_TAB + (m >> 4) * 8);
  return v & u32x4v{lo[0], lo[1], hi[0], hi[1]};
}
template <int N>
__device__ __forceinline__ void barrier_vmt() {  // barrier after all but the N youngest vector-memory ops
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"i"(N) : "memory");
}

#if ASR_DEEP_TRACE  // diagnostic: per-step timestamps of workgroup 0 (waves 0, 4, 7)
__device__ unsigned long long g_trace[3][160][4];
#define ASR_TRACE(role, t, which)                                     \
  if (blockIdx.x == 0 && (threadIdx.x & 63) == 0 && (t) < 160) {      \
    unsigned long long tt_ = __builtin_amdgcn_s_memtime();            \
    unsigned lo_ = (unsigned)tt_, hi_ = (unsigned)(tt_ >> 32);        \
    asm volatile("v_mov_b32 %0, %0\n\tv_mov_b32 %1, %1" : "+v"(lo_), "+v"(hi_)); \
    g_trace[role][t][which] = ((unsigned long long)hi_ << 32) | lo_;  \
  }
#else
#define ASR_TRACE(role, t, which)
#endif

// The workgroup's layer steps in order: segments sg, its images n = b, b+P, ..,
// layers ltop(sg) - k.  Every prefetch (x two steps ahead, masks two steps
// ahead, the next image's dx) follows this stream across image and segment
// boundaries; past the last step it repeats the last one (harmless reloads).
struct Pos {
  int sg, n, k;
};
__device__ __forceinline__ int seg_top(int L, int sg) { return L - 1 - sg * KSEG; }
__device__ __forceinline__ int seg_len(int L, int sg) { return min(KSEG, L - sg * KSEG); }
__device__ __forceinline__ Pos pos_next(Pos s, int L, int N, int P, int b) {
  if (s.k + 1 < seg_len(L, s.sg)) return {s.sg, s.n, s.k + 1};
  if (s.n + P < N) return {s.sg, s.n + P, 0};
  if ((s.sg + 1) * KSEG < L) return {s.sg + 1, b, 0};
  return s;
}
__device__ __forceinline__ int pos_layer(Pos s, int L) { return seg_top(L, s.sg) - s.k; }

template <bool GAMMA>
__global__ __launch_bounds__(64 * NWB, 1) void k_bwd16_fused(bf16* __restrict__ dbufA, bf16* __restrict__ dbufB,
                                                            const bf16* __restrict__ xs, long x_stride,
                                                            const uint8_t* __restrict__ masks, long mask_stride,
                                                            const bf16* __restrict__ wpack, float h, float two_gamma,
                                                            int N, int L, float* __restrict__ slabs, int PS) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, lx = lane & 15, q = lx >> 2, p = lx & 3;
  const int P = gridDim.x, b = blockIdx.x;
  // dz tiles, their zero row, the x tiles and the third x row block (halos stay zero)
  for (int i = tid; i < L_M / 16; i += 64 * NWB) ((uint4*)lds)[i] = make_uint4(0, 0, 0, 0);
  for (int i = tid; i < (L_TOTAL - L_E) / 16; i += 64 * NWB) ((uint4*)(lds + L_E))[i] = make_uint4(0, 0, 0, 0);
  if (tid < 16) {
    u32x2 e;
#pragma unroll
    for (int d = 0; d < 2; ++d) e[d] = ((tid >> (2 * d)) & 1 ? 0xffffu : 0u) | ((tid >> (2 * d + 1)) & 1 ? 0xffff0000u : 0u);
    *(u32x2*)(lds + L_TAB + tid * 8) = e;
  }
  __syncthreads();
  const int nseg = (L + KSEG - 1) / KSEG;

  if (wave < NDG) {
    // ------------------------------ dgrad waves ------------------------------
    const int r0 = wave * RPB;
    const float hs2g = h * two_gamma;
    const unsigned bF = (unsigned)(r0 * ROWB) + swz(lx + (g >> 1), g & 1);
    const unsigned bG = (unsigned)((r0 + (g >> 1)) * ROWB) + swz(lx + 2, g & 1);
    const int px = lx + 16 * (g & 1), cg = g >> 1;
    const unsigned oT = (unsigned)((r0 + 1) * ROWB) + swz(px + 1, cg);
    const unsigned oG = (unsigned)(((r0 * W + px) * C + 8 * cg) * 2);
    const unsigned oM = (unsigned)((r0 * W + px) * 2 + cg);
    unsigned wo[KS];
    wt_offsets(lane, wo);
    int t = 0;  // layer steps so far: buffer parity (identical count in every role)
    // dx_{l+1} of the wave's pixels (regrouped chunks), fp32 between layers; at an
    // image's segment top the bf16 dx from HBM sits raw in the first two pairs
    f32x2 dxf[RPB][4];
    auto raw_load = [&](int j, const unsigned char* src) {
      const u32x4v v = *(const u32x4v*)src;
      dxf[j][0] = (f32x2){__uint_as_float(v[0]), __uint_as_float(v[1])};
      dxf[j][1] = (f32x2){__uint_as_float(v[2]), __uint_as_float(v[3])};
    };
#pragma unroll
    for (int j = 0; j < RPB; ++j) raw_load(j, (const unsigned char*)dbufA + (long)b * IMG * 2 + oG + j * ROW_G);
    barrier_lds();  // prologue: wave 7's DMA of the first x / masks
    for (int sg = 0; sg < nseg; ++sg) {
      const int ltop = L - 1 - sg * KSEG, kcount = min(KSEG, ltop + 1);
      unsigned char* dout = (unsigned char*)((sg & 1) ? dbufA : dbufB);
      for (int n = b; n < N; n += P) {
        const long img = (long)n * IMG * 2;
        // dzm_ltop = dx & mask_ltop into dz tile t
        {
          const unsigned char* mt = lds + L_M + (t & 1) * MB;
#pragma unroll
          for (int j = 0; j < RPB; ++j) {
            const u32x4v w = {__float_as_uint(dxf[j][0].x), __float_as_uint(dxf[j][0].y), __float_as_uint(dxf[j][1].x),
                              __float_as_uint(dxf[j][1].y)};
            *(u32x4v*)(lds + L_Z + (t & 1) * TILE + oT + j * ROWB) = mask_bf16x8(lds, w, mt[oM + j * 64]);
#pragma unroll
            for (int d = 0; d < 4; ++d) dxf[j][d] = (f32x2){lo_f(w[d]), hi_f(w[d])};
          }
        }
        bf16x8 A0[KS], A1[KS];
        load_wt(wpack + (long)ltop * WSTRIDE, wo, A0);
        barrier_lds();
        // one layer step; LAST: the image's last layer of the segment (dx out, next
        // image's dx in); A this layer's W^T, An receives the next layer's
        auto step = [&](int k, auto last_c, bf16x8 (&A)[KS], bf16x8 (&An)[KS]) {
          constexpr bool LAST = decltype(last_c)::value;
          if (wave == 0) ASR_TRACE(0, t, 0);
          const int l = ltop - k;
          const unsigned char* zt = lds + L_Z + (t & 1) * TILE;
          unsigned char* zn = lds + L_Z + ((t + 1) & 1) * TILE;
          const unsigned char* mn = lds + L_M + ((t + 1) & 1) * MB;  // mask_{l-1}
          load_wt(wpack + (long)max(l - 1, 0) * WSTRIDE, wo, An);      // branch-free prefetch
          const Pos nx = pos_next({sg, n, k}, L, N, P, b);  // the next image's (or segment's) top
          const unsigned char* dnext =
              (const unsigned char*)((nx.sg & 1) ? dbufB : dbufA) + (long)nx.n * IMG * 2;
          constexpr int NS = NDG == 8 ? 3 : 4;  // 3 slots at 3 waves per SIMD (VGPR budget)
          FragT<NS> fr;
#pragma unroll
          for (int R = 0; R < 3; ++R) fr.load(zt, bF, bG, R);
#pragma unroll
          for (int j = 0; j < RPB; ++j) {
            if (NS == 4 && j + 3 <= RPB + 1) fr.load(zt, bF, bG, j + 3);
            f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
            row_mfma(A, fr.F[j % NS], fr.F[(j + 1) % NS], fr.F[(j + 2) % NS], fr.G[j % NS], fr.G[(j + 2) % NS], acc);
            if (NS == 3 && j + 3 <= RPB + 1) fr.load(zt, bF, bG, j + 3);
            u32x4v zw;
            if constexpr (GAMMA) zw = *(const u32x4v*)(zt + oT + j * ROWB);  // dzm_l of the lane's chunk
            float c[8];
            regroup(acc[0], acc[1], c);
            u32x4v ow;
#pragma unroll
            for (int d = 0; d < 4; ++d) {
              f32x2 v = pk_fma(-h, (f32x2){c[2 * d], c[2 * d + 1]}, dxf[j][d]);
              if constexpr (GAMMA) v = pk_fma(hs2g, (f32x2){lo_f(zw[d]), hi_f(zw[d])}, v);
              dxf[j][d] = v;
              ow[d] = pk_bf16(v.x, v.y);
            }
            if constexpr (!LAST) {
              *(u32x4v*)(zn + oT + j * ROWB) = mask_bf16x8(lds, ow, mn[oM + j * 64]);
            } else {
              *(u32x4v*)(dout + img + oG + j * ROW_G) = ow;
              raw_load(j, dnext + oG + j * ROW_G);
            }
          }
          if (wave == 0) ASR_TRACE(0, t, 1);
          ++t;
          barrier_lds();  // dz_{l-1} complete, dz_l / x_l consumed
        };
        int k = 0;
        for (; k + 2 < kcount; k += 2) {  // the two register sets alternate
          step(k, std::false_type{}, A0, A1);
          step(k + 1, std::false_type{}, A1, A0);
        }
        if (k + 1 < kcount) {
          step(k, std::false_type{}, A0, A1);
          step(k + 1, std::true_type{}, A1, A0);
        } else {
          step(k, std::true_type{}, A0, A1);
        }
      }
      __syncthreads();  // segment end (slabs written by the wgrad waves and wave 7)
      __syncthreads();
    }
  } else if (wave < NDG + 3) {
    // ------------------------------ wgrad waves ------------------------------
    const int kx = wave - NDG;
    unsigned tx2[2], tz2[2];  // tr-read lane offsets: pixel 8g + 4*(hh ^ (g&1)) + q, channels 4p..4p+3
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int pix = 8 * g + 4 * (hh ^ (g & 1)) + q;
      tx2[hh] = (unsigned)(pix * 32 + 8 * p);
      tz2[hh] = swz(pix + 1, p >> 1) + 8 * (p & 1);
    }
    f32x4 acc[KSEG][3];
    // one layer's weight gradient for tap column kx into a[ky] (ky = 0..2): the x
    // fragment of image row ir-1 feeds output rows ir - ky; reads run DEPTH rows
    // ahead of the MFMAs
    auto wgrad_layer = [&](f32x4 (&a)[3], int tt) {
      constexpr int DEPTH = WDEPTH;
      const int par = tt & 1;
      const unsigned char* xt = lds + L_X + par * XT + kx * 32 - ROWB;  // + ir*ROWB: image row ir-1 < XS
      const unsigned char* xh = lds + xhi_base(tt) - XS * ROWB + kx * 32 - ROWB;  // image rows >= XS
      const unsigned char* zt = lds + L_Z + par * TILE + ROWB;          // + d*ROWB: output row d
      auto xrow = [&](int ir) { return (ir - 1 < XS ? xt : xh) + ir * ROWB; };
      bf16x8 Aq[DEPTH + 1], Bq[DEPTH + 1];
      const bf16x8 Bz = tr2(zt, tz2);
#pragma unroll
      for (int d = 1; d <= DEPTH; ++d) {
        Aq[d % (DEPTH + 1)] = tr2(xrow(d), tx2);
        if (d < H) Bq[d % (DEPTH + 1)] = tr2(zt + d * ROWB, tz2);
      }
      bf16x8 Bm1 = Bz, Bm2 = Bz;
#pragma unroll
      for (int ir = 1; ir <= H; ++ir) {
        if (ir + DEPTH <= H) {
          Aq[(ir + DEPTH) % (DEPTH + 1)] = tr2(xrow(ir + DEPTH), tx2);
          if (ir + DEPTH < H) Bq[(ir + DEPTH) % (DEPTH + 1)] = tr2(zt + (ir + DEPTH) * ROWB, tz2);
        }
        const bf16x8 Ax = Aq[ir % (DEPTH + 1)];
        if (ir < H) a[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ax, Bq[ir % (DEPTH + 1)], a[0], 0, 0, 0);  // ky=0
        a[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ax, Bm1, a[1], 0, 0, 0);  // ky=1: output row ir-1
        if (ir >= 2) a[2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ax, Bm2, a[2], 0, 0, 0);  // ky=2: row ir-2
        Bm2 = Bm1;
        if (ir < H) Bm1 = Bq[ir % (DEPTH + 1)];
      }
    };
    int t = 0;
    barrier_lds();  // prologue
    for (int sg = 0; sg < nseg; ++sg) {
      const int ltop = L - 1 - sg * KSEG, kcount = min(KSEG, ltop + 1);
#pragma unroll
      for (int k = 0; k < KSEG; ++k)
#pragma unroll
        for (int e = 0; e < 3; ++e) acc[k][e] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int n = b; n < N; n += P) {
        barrier_lds();  // dzm_ltop written
        for (int k = 0; k < kcount; ++k) {
          if (wave == NDG) ASR_TRACE(1, t, 0);
          static_for<0, KSEG>([&](auto kc) {
            if (k == decltype(kc)::value) wgrad_layer(acc[decltype(kc)::value], t);
          });
          if (wave == NDG) ASR_TRACE(1, t, 1);
          ++t;
          barrier_lds();
        }
      }
      // segment end: dW of each layer straight from the accumulators (complete sums)
      __syncthreads();
      static_for<0, KSEG>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        if (k >= kcount) return;
        float* slab = slabs + ((long)(ltop - k) * PS + b) * ES;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int e = 0; e < 4; ++e) slab[((3 * ky + kx) * 16 + 4 * g + e) * 16 + lx] = h * acc[k][ky][e];
      });
      __syncthreads();
    }
  } else {
    // -------------------------- x / mask staging wave (7) --------------------------
    // x of the step after next: rows 0..XS-1 by global loads into registers (a
    // third x buffer), written to the free LDS x tile one step later; rows XS..
    // by LDS-DMA into the rotating third row block; so every x load has about
    // two layer steps to land.  Masks likewise through registers (three steps
    // ahead of the dgrad epilogue that reads them); db of each layer on MFMA.
    constexpr int HS = XS;
    const unsigned lb = lds_u32(lds);  // LDS byte address of the dynamic allocation
    u32x4v st[HS];
    unsigned tz2[2];  // dz tr-read lane offsets (as the wgrad waves)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) tz2[hh] = swz(8 * g + 4 * (hh ^ (g & 1)) + q + 1, p >> 1) + 8 * (p & 1);
    // db on MFMA: D = ones(16 x 32 pixels) x dzm(32 pixels x 16 o), one row per
    // MFMA, every D row = the per-channel sum (fixed order); added per image into
    // the segment's db sums in LDS (one lane per channel: deterministic)
    float* dbl = (float*)(lds + L_DB);
    const bf16x8 ones = {(bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f};
    auto db_layer = [&](f32x4& a, int par) {
      const unsigned char* zt = lds + L_Z + par * TILE + ROWB;
      bf16x8 B[4];
#pragma unroll
      for (int d = 0; d < 3; ++d) B[d] = tr2(zt + d * ROWB, tz2);
#pragma unroll
      for (int d = 0; d < H; ++d) {
        if (d + 3 < H) B[(d + 3) & 3] = tr2(zt + (d + 3) * ROWB, tz2);
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, B[d & 3], a, 0, 0, 0);
      }
    };
    auto load_x = [&](Pos s) {
      const unsigned char* src = (const unsigned char*)(xs + pos_layer(s, L) * x_stride + (long)s.n * IMG) + lane * 16;
#pragma unroll
      for (int j = 0; j < HS; ++j) st[j] = *(const u32x4v*)(src + j * ROW_G);
    };
    auto write_x = [&](int par) {
      unsigned char* dst = lds + L_X + par * XT + 32 + lane * 16;
#pragma unroll
      for (int j = 0; j < HS; ++j) *(u32x4v*)(dst + j * ROWB) = st[j];
    };
    auto dma_x = [&](Pos s, int j0, int tt) {  // rows j0.. of step tt's x (rows < XS: tile tt & 1)
      const unsigned char* xsrc = (const unsigned char*)(xs + pos_layer(s, L) * x_stride + (long)s.n * IMG);
      const unsigned hb = lb + xhi_base(tt) - XS * ROWB + 32, lo = lb + L_X + (tt & 1) * XT + 32;
      for (int j = j0; j < H; ++j) dma16_at(xsrc + j * ROW_G + lane * 16, (j < XS ? lo : hb) + j * ROWB);
    };
    u32x4v mst[2];  // a mask (2 KiB) staged in registers, as the x rows
    auto load_m = [&](Pos s) {
      const unsigned char* src = masks + pos_layer(s, L) * mask_stride + (long)s.n * MB + lane * 16;
      mst[0] = *(const u32x4v*)src;
      mst[1] = *(const u32x4v*)(src + 1024);
    };
    auto write_m = [&](int par) {
      *(u32x4v*)(lds + L_M + par * MB + lane * 16) = mst[0];
      *(u32x4v*)(lds + L_M + par * MB + 1024 + lane * 16) = mst[1];
    };
    auto dma_m = [&](Pos s, int par) {
      const uint8_t* msrc = masks + pos_layer(s, L) * mask_stride + (long)s.n * MB;
      for (int j = 0; j < 2; ++j) dma16_at(msrc + j * 1024 + lane * 16, lb + L_M + par * MB + j * 1024);
    };
    int t = 0;
    {  // prologue: the first step's x and masks, the next step's x and mask
      const Pos p0 = {0, b, 0}, p1 = pos_next(p0, L, N, P, b), p2 = pos_next(p1, L, N, P, b);
      dma_x(p0, 0, 0);
      dma_m(p0, 0);
      dma_m(p1, 1);
      dma_x(p1, XS, 1);
      load_x(p1);
      load_m(p2);
      barrier_vmt<H + 2>();  // the first x and masks landed; the next ones keep flying
    }
    for (int sg = 0; sg < nseg; ++sg) {
      const int ltop = L - 1 - sg * KSEG, kcount = min(KSEG, ltop + 1);
      for (int i = lane; i < KSEG * C; i += 64) dbl[i] = 0.f;
      for (int n = b; n < N; n += P) {
        barrier_lds();  // dzm_ltop written
        for (int k = 0; k < kcount; ++k) {
          ASR_TRACE(2, t, 0);
          const Pos n1 = pos_next({sg, n, k}, L, N, P, b), n2 = pos_next(n1, L, N, P, b),
                    n3 = pos_next(n2, L, N, P, b);
          write_x((t + 1) & 1);  // x of the next step
          write_m(t & 1);        // mask of the step after next (read by the next step's dgrad epilogue)
#if ASR_DEEP_TRACE
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
          ASR_TRACE(2, t, 2);
          dma_x(n2, XS, t + 2);  // upper x rows of the step after next
          load_x(n2);
          load_m(n3);
          {
            f32x4 a = {0.f, 0.f, 0.f, 0.f};
            db_layer(a, t & 1);
            if (g == 0) dbl[k * C + lx] += a[0];
          }
          ASR_TRACE(2, t, 3);
#if ASR_DEEP_TRACE
          asm volatile("s_waitcnt vmcnt(34)" ::: "memory");  // trace the x DMA landing, not its issue
#endif
          ASR_TRACE(2, t, 1);
          ++t;
          barrier_vmt<H + 2>();  // the previous step's x DMA landed; this step's loads keep flying
        }
      }
      __syncthreads();
      for (int k = 0; k < kcount; ++k)
        if (g == 0) slabs[((long)(ltop - k) * PS + b) * ES + 9 * C * C + lx] = h * dbl[k * C + lx];
      for (int k = 0; k < kcount; ++k)  // padding slabs of the 32-slab reduction groups
        for (int j = P + b; j < PS; j += P) {
          float* zs = slabs + ((long)(ltop - k) * PS + j) * ES;
          for (int i = lane; i < ES; i += 64) zs[i] = 0.f;
        }
      __syncthreads();
    }
  }
}
}  // namespace deep

bool deep16_supported(int H, int W, int C) { return C == deep::C && H == deep::H && W == deep::W; }

// L Euler blocks in one launch (see k_fwd16_fused).  bias: layer l's at
// bias + l*bias_stride; wpack: asr_theta_to_w's bf16 output for the L layers.
int deep16_forward(const void* x0, void* y0, long y_stride, uint8_t* mask0, long mask_stride, const void* wpack,
                   const float* bias, long bias_stride, float h, int N, int L, bool store_all, hipStream_t s) {
  if (L < 1 || N < 1) return fail(ASR_E_ARG, "deep16_forward: bad N=%d L=%d", N, L);
  int cus = cu_count();
  if (cus <= 0) cus = 256;
  const int grid = std::max(1, std::min(N, 2 * cus));
  const size_t lds = 2 * (size_t)deep::TILE + deep::ROWB;
#define ASR_FWD16(SA, MK)                                                                                        \
  hipLaunchKernelGGL((deep::k_fwd16_fused<SA, MK>), dim3(grid), dim3(64 * deep::NWAVE), lds, s, (const bf16*)x0, \
                     (bf16*)y0, y_stride, mask0, mask_stride, (const bf16*)wpack, bias, bias_stride, h, N, L)
  if (store_all) {
    if (mask0) ASR_FWD16(true, true);
    else ASR_FWD16(true, false);
  } else {
    if (mask0) ASR_FWD16(false, true);
    else ASR_FWD16(false, false);
  }
#undef ASR_FWD16
  ASR_LAUNCH_CHECK("k_fwd16_fused");
  return ASR_OK;
}

#if ASR_DEEP_TRACE
extern "C" int asr_debug_deep16_trace(void* dst, size_t bytes) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(deep::g_trace), bytes) == hipSuccess ? 0 : -1;
}
#endif

int deep16_slab_rows(int N) {
  int cus = cu_count();
  if (cus <= 0) cus = 256;
  const int P = std::max(1, std::min(N, cus));
  return (P + 31) / 32 * 32;
}

size_t deep16_slab_bytes(int N, int L) { return (size_t)L * deep16_slab_rows(N) * deep::ES * sizeof(float); }

// Backward of deep16_forward over all L layers (see k_bwd16_fused).  dbufA
// holds dL/dx_L on entry; dx_0 ends in dbufA or dbufB (*dx0_in_b).  slabs:
// deep16_slab_bytes(N, L) bytes, layout [L][slab_rows][ES].
int deep16_backward(void* dbufA, void* dbufB, const void* xs, long x_stride, const uint8_t* masks, long mask_stride,
                    const void* wpack, float h, float two_gamma, int N, int L, float* slabs, int* slab_rows,
                    int* dx0_in_b, hipStream_t s) {
  if (L < 1 || N < 1) return fail(ASR_E_ARG, "deep16_backward: bad N=%d L=%d", N, L);
  int cus = cu_count();
  if (cus <= 0) cus = 256;
  const int P = std::max(1, std::min(N, cus));
  const int PS = deep16_slab_rows(N);
  auto kern = two_gamma != 0.f ? deep::k_bwd16_fused<true> : deep::k_bwd16_fused<false>;
  hipLaunchKernelGGL(kern, dim3(P), dim3(64 * deep::NWB), (size_t)deep::L_TOTAL, s, (bf16*)dbufA, (bf16*)dbufB,
                     (const bf16*)xs, x_stride, masks, mask_stride, (const bf16*)wpack, h, two_gamma, N, L, slabs, PS);
  ASR_LAUNCH_CHECK("k_bwd16_fused");
  *slab_rows = PS;
  *dx0_in_b = ((L + deep::KSEG - 1) / deep::KSEG) & 1;
  return ASR_OK;
}

}  // namespace asr
