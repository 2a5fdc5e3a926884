// Persistent, LDS-DMA-pipelined bf16 kernels of the antisymmetric Euler block
// (gfx950): forward, and a FUSED backward (dgrad + wgrad + db in one pass).
//
// Reference operator: Conv2DAntisymmetric3By3.call (tf.nn.conv2d SAME NHWC +
// bias, layers/tfkeras_layer_Conv2DAntisymmetric3By3.py:157-171) inside
// single_layer_identity_block (relu, h*, +input: models/tfkeras_resnets.py:69-92)
// and its autodiff (training/training.py:300).
//
// Work item = one band of BR output rows of one image.  One 512-thread
// workgroup per CU walks a contiguous run of items (consecutive bands of the
// same images, so halo rows are L2 hits).  The input rows of item i+1 are
// copied HBM -> LDS by global_load_lds (no VGPR staging) while item i is
// computed; the XOR swizzle of the LDS image is applied on the per-lane
// SOURCE address (the DMA writes 1 KiB lane-linear), halo columns are zeroed
// once, rows outside the image come from a zero page.
//
// Math (implicit GEMM on v_mfma_f32_16x16x32_bf16, kappa = tap*C + i):
//   forward  Z^T[o][p]  = sum_kappa W^T[o][kappa] X[p][kappa]      (A = W^T in VGPRs)
//   dgrad    (A dz)     : the same GEMM on dz = h*dy*mask, because
//                         A^T = -A + 2*gamma*I for the assembled W:
//                         dx = dy - A dz + 2*gamma*dz
//   wgrad    dW[kappa][o] = sum_p X[p + s(tap)][i] dz[p][o]          (K = pixels;
//                         both operands read with ds_read_b64_tr_b16)
// In the fused backward, waves 0-3 own the dgrad (W fragments resident in
// VGPRs) and waves 4-7 own the wgrad (the dW tile set resident in
// accumulators for the workgroup's whole run); both consume the same LDS
// images of dz (computed once per item from dy and the relu mask) and x.
#include <stdlib.h>

#include <type_traits>

#include "asr_common.h"
#include "asr_device.h"

// Measured settings (each an A/B of whole steps in the commit log; the other arms were removed in
// round 6 and stay in git history).  The v1 backward (C = 16 / 32, RK2 stages): 75 % of its prefetch
// DMAs issued by the dgrad waves, inside their k-steps.  The v2/v3 backward's convert: relu-mask
// expansion from a 4 KiB LDS table.  The forward pipe: y as 16-B stores; halo rows of a band that
// continues the previous band's image copied in LDS.
constexpr int kBwdDgradDmaPct = 75;
constexpr int kFwd3Wgs = 3;  // k_fwd3 workgroups per CU (grid = min(bands, 3 x CUs))
// k_bwd3 wgrad waves: DMA pieces issued right after the barrier, the rest one per row (A/B: spreading them
// lengthened the MFMA phase as much as it saved; the stacks: all at once 16 vs 9 +0.3-0.5 %, 4 -0.7 %)
constexpr int kBwd3Dma0 = 16;

namespace asr {

namespace blk {

// Diagnostic build only (-DASR_STAMP_BUILD=1, cdna_hip_programming.md §7
// in-kernel stamps): s_memtime at phase boundaries of the fused backward,
// lane 0 of waves 0 (dgrad) and 4 (wgrad), into a buffer nothing else reads.
#ifndef ASR_STAMP_BUILD
#define ASR_STAMP_BUILD 0
#endif
#if ASR_STAMP_BUILD
constexpr int kStampBands = 16, kStampSlots = 8;
__device__ unsigned long long g_stamps[512][2][kStampBands][kStampSlots];
#define ASR_STAMP(band, slot)                                                                      \
  do {                                                                                             \
    if ((wave == 0 || wave == 4) && (band) < kStampBands) {                                        \
      unsigned long long _t;                                                                       \
      __builtin_amdgcn_sched_barrier(0);                                                           \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                   \
      __builtin_amdgcn_sched_barrier(0);                                                           \
      if (lane == 0) g_stamps[blockIdx.x][wave >> 2][(band)][(slot)] = _t;                         \
    }                                                                                              \
  } while (0)
#else
#define ASR_STAMP(band, slot) \
  do {                        \
  } while (0)
#endif

enum { FWD_EULER = 0, FWD_CONV = 1, BWD_EULER = 2, BWD_CONV = 3 };

// Diagnostic build only (-DASR_BLK_TRACE=1): s_memtime stamps per band of
// workgroup 0 in k_fwd3 (kernel 0, wave 0) and k_bwd3 (kernel 1, role 0 =
// dgrad wave 0, role 1 = wgrad wave 4), and the clock probe pair (s_memtime,
// s_memrealtime) at the start and end of wave 0 in every workgroup; into
// buffers nothing else reads (asr_debug_blk_trace).
#ifndef ASR_BLK_TRACE
#define ASR_BLK_TRACE 0
#endif
#if ASR_BLK_TRACE
constexpr int kTrBands = 40, kTrSlots = 8;
__device__ unsigned long long g_btrace[2][2][kTrBands][kTrSlots];
__device__ unsigned long long g_bclock[2][1024][4];
// every workgroup at every block switch of k_bwd3_stack (the first band of block l), [wg][l][slot]:
// 0 wgrad wave 4 before the done[] poll, 1 after the poll and fence, 2 after its band barrier,
// 3 dgrad wave 0 before its band barrier, 4 after it (s_memtime: durations inside a workgroup);
// 5 / 6 s_memrealtime at slots 0 / 2 (100 MHz, one time base for every workgroup)
constexpr int kSwBlocks = 128, kSwSlots = 7;
__device__ unsigned long long g_bswitch[256][kSwBlocks][kSwSlots];
__device__ __forceinline__ void tr_store(unsigned long long* p, unsigned long long t) {
  unsigned lo = (unsigned)t, hi = (unsigned)(t >> 32);
  asm volatile("v_mov_b32 %0, %0\n\tv_mov_b32 %1, %1" : "+v"(lo), "+v"(hi));  // vector store
  *p = ((unsigned long long)hi << 32) | lo;
}
#define ASR_BTR(kern, role, band, slot)                                                         \
  do {                                                                                          \
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0 && (band) < kTrBands)                        \
      tr_store(&g_btrace[kern][role][band][slot], __builtin_amdgcn_s_memtime());                \
  } while (0)
#define ASR_BSW(l, slot, rt)                                                                   \
  do {                                                                                         \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 256 && (l) < kSwBlocks)                       \
      tr_store(&g_bswitch[blockIdx.x][l][slot],                                                \
               (rt) ? __builtin_amdgcn_s_memrealtime() : __builtin_amdgcn_s_memtime());       \
  } while (0)
#define ASR_BCLK(kern, which)                                                                    \
  do {                                                                                           \
    if (threadIdx.x == 0 && blockIdx.x < 1024) {                                                 \
      tr_store(&g_bclock[kern][blockIdx.x][2 * (which)], __builtin_amdgcn_s_memtime());          \
      tr_store(&g_bclock[kern][blockIdx.x][2 * (which) + 1], __builtin_amdgcn_s_memrealtime());  \
    }                                                                                            \
  } while (0)
#else
#define ASR_BSW(l, slot, rt) \
  do {                       \
  } while (0)
#define ASR_BTR(kern, role, band, slot) \
  do {                                  \
  } while (0)
#define ASR_BCLK(kern, which) \
  do {                        \
  } while (0)
#endif

template <int C>
struct Geo {
  static constexpr int NQ = C / 8;              // 16-byte chunks per pixel
  static constexpr int OT = C / 16;             // 16-channel tiles
  static constexpr int KS = (9 * C + 31) / 32;  // 32-deep k-steps of the conv GEMM
  static constexpr int OSPLIT = (C == 64) ? 2 : 1;
  static constexpr int OTW = OT / OSPLIT;       // o-tiles per conv wave
  static constexpr int MT = 9 * C / 16;         // wgrad m-tiles
  static constexpr int MTW = 9;                 // wgrad m-tiles per wave
  static constexpr int TG = MT / MTW;           // wgrad tile groups
  static constexpr int KSPLIT = 4 / TG;         // wgrad waves sharing a tile group
  static constexpr int PPI = 512 / C;           // pixels per 1 KiB DMA instruction
  __device__ __forceinline__ static int swz(int col) {
    if constexpr (C == 64) return col & 7;
    else if constexpr (C == 32) return (col >> 1) & 3;
    else return 0;
  }
};

template <int C>
__device__ __forceinline__ int toff(int row, int col, int q, int TW) {
  return ((row * TW + col) * Geo<C>::NQ + (q ^ Geo<C>::swz(col))) * 16;
}

// DMA image rows [gy0, gy0+nrows) of image n (rows outside [0,H) -> zeros) into
// tile rows [0, nrows), interior columns 1..W.  One instruction = PPI pixels.
// The lane's source offset inside a PPI-pixel segment does not depend on the
// segment (swz(col) only sees col mod 8 / mod 16, and PPI is a multiple of
// that), so per instruction only a wave-uniform base changes.
template <int C, int W>
__device__ __forceinline__ int dma_lane_off(int lane) {
  using G = Geo<C>;
  const int pl = lane / G::NQ, p = lane % G::NQ;
  return pl * C + (p ^ G::swz(1 + pl)) * 8;  // elements
}

// The loops below run on a wave-uniform index (readfirstlane), so they are
// scalar loops: per instruction only an SGPR base (row start or the zero
// page) and M0 change; the per-lane part is one 32-bit offset.
//
// One instruction j of a row stream: image rows [gy0, gy0+nrows) of image n
// (rows outside [0,H) -> zeros) into tile rows [0, nrows), interior columns.
template <int C, int W>
__device__ __forceinline__ void dma_row_instr(const bf16* __restrict__ src, unsigned char* tile, int n, int gy0, int j,
                                              int H, unsigned loff) {
  using G = Geo<C>;
  constexpr int TW = W + 2, NQ = G::NQ, PPI = G::PPI, IPR = W / PPI;
  const int r = (unsigned)j / IPR, seg = (unsigned)j % IPR;  // wave-uniform
  const int gy = gy0 + r;
  const unsigned char* base = ((unsigned)gy < (unsigned)H)
                                  ? (const unsigned char*)src + ((long)n * H + gy) * (W * C * 2) + seg * (PPI * C * 2)
                                  : (const unsigned char*)g_zero_page;
  dma16(base + loff, tile + ((r * TW + 1 + seg * PPI) * NQ) * 16);
}

// dma_row_instr to a tile at an LDS byte address (no generic -> LDS pointer cast: its
// null check trips a ROCm 7.2 codegen bug in the register-tight stacked backward)
template <int C, int W>
__device__ __forceinline__ void dma_row_instr_at(const bf16* __restrict__ src, unsigned tile, int n, int gy0, int j,
                                                 int H, unsigned loff) {
  using G = Geo<C>;
  constexpr int TW = W + 2, NQ = G::NQ, PPI = G::PPI, IPR = W / PPI;
  const int r = (unsigned)j / IPR, seg = (unsigned)j % IPR;  // wave-uniform
  const int gy = gy0 + r;
  const unsigned char* base = ((unsigned)gy < (unsigned)H)
                                  ? (const unsigned char*)src + ((long)n * H + gy) * (W * C * 2) + seg * (PPI * C * 2)
                                  : (const unsigned char*)g_zero_page;
  dma16_at(base + loff, tile + (unsigned)((r * TW + 1 + seg * PPI) * NQ) * 16u);
}

// Image row gy (zeros outside [0, H)) into a tile row: its W / PPI = 4 pieces in
// one dma16x4_at (the lane's swizzled source offset is the same for every
// piece: the swizzle is segment-invariant).  tile_row = the tile row's LDS byte address.
template <int C, int W>
__device__ __forceinline__ void dma_row_whole_at(const bf16* __restrict__ src, unsigned tile_row, int n, int gy, int H,
                                                 unsigned loff) {
  using G = Geo<C>;
  constexpr int NQ = G::NQ, PPI = G::PPI;
  static_assert(W / PPI == 4 && PPI * C * 2 == 1024 && PPI * NQ * 16 == 1024, "whole-row DMA: four 1 KiB pieces");
  const unsigned char* base = ((unsigned)gy < (unsigned)H)
                                  ? (const unsigned char*)src + ((long)n * H + gy) * (W * C * 2)
                                  : (const unsigned char*)g_zero_page;
  dma16x4_at(base + loff, tile_row + (unsigned)(NQ * 16));
}

template <int C, int W>
__device__ __forceinline__ void dma_rows(const bf16* __restrict__ src, unsigned char* tile, int n, int gy0,
                                         int nrows, int H, int wave, int nwaves, int lane) {
  using G = Geo<C>;
  constexpr int PPI = G::PPI, IPR = W / PPI;
  static_assert(W % PPI == 0, "image width must be a multiple of the DMA pixel group");
  static_assert(PPI % 16 == 0 || (PPI % 8 == 0 && C == 64), "segment-invariant swizzle");
  const unsigned loff = (unsigned)dma_lane_off<C, W>(lane) * 2u;  // bytes, < 1 KiB
  for (int j = __builtin_amdgcn_readfirstlane(wave); j < nrows * IPR; j += nwaves)
    dma_row_instr<C, W>(src, tile, n, gy0, j, H, loff);
}

// One 1 KiB chunk j of the relu-mask bytes of rows [gy0, gy0+nrows) (W*C/8
// bytes per row) into a lane-linear LDS array (bytes outside the image ->
// zeros).  The band's rows are contiguous in memory; only chunks that reach
// outside the image take the per-lane select.
template <int C, int W>
__device__ __forceinline__ void dma_mask_instr(const uint8_t* __restrict__ mask, unsigned char* mt, int n, int gy0,
                                               int nrows, int j, int H, int lane) {
  constexpr int RB = W * C / 8;  // bytes per image row
  const int total = nrows * RB;
  const long band0 = ((long)n * H + gy0) * RB;
  const int lo = max(0, -gy0) * RB, hi = (min(H, gy0 + nrows) - gy0) * RB;  // valid bytes of the band
  const int b0 = j * 1024, b = b0 + lane * 16;
  const void* s;
  if (b0 >= lo && b0 + 1024 <= hi && b0 + 1024 <= total)  // whole chunk valid (uniform)
    s = (const void*)(mask + band0 + b);
  else
    s = (b >= lo && b < hi && b < total) ? (const void*)(mask + band0 + b) : (const void*)(g_zero_page + lane);
  dma16(s, mt + b0);
}

template <int C, int W>
__device__ __forceinline__ void dma_mask_rows(const uint8_t* __restrict__ mask, unsigned char* mt, int n, int gy0,
                                              int nrows, int H, int wave, int nwaves, int lane) {
  const int total = nrows * (W * C / 8);
  for (int j = __builtin_amdgcn_readfirstlane(wave); j * 1024 < total; j += nwaves)
    dma_mask_instr<C, W>(mask, mt, n, gy0, nrows, j, H, lane);
}

// zero the halo columns (0 and W+1) of a tile with `rows` rows
template <int C, int W>
__device__ __forceinline__ void zero_halo_cols(unsigned char* tile, int rows, int tid, int nthreads) {
  constexpr int TW = W + 2, NQ = Geo<C>::NQ;
  for (int i = tid; i < rows * 2 * NQ; i += nthreads) {
    const int q = i % NQ, side = (i / NQ) & 1, r = i / (2 * NQ);
    *(uint4*)(tile + toff<C>(r, side ? W + 1 : 0, q, TW)) = make_uint4(0, 0, 0, 0);
  }
}

// Per-lane LDS offsets of the conv GEMM's B fragments.  k-step ks covers
// kappa = 32*ks + 8*g + j (g = lane>>4): for C >= 32 that is tap 32*ks/C and
// chunk qb + g (qb = (32*ks % C)/8), so only the 3 column shifts x the C/32
// chunk bases are lane-dependent (3 or 6 VGPRs); the tap row and the pixel
// tile become ds_read immediates.  For C = 16 the tap itself depends on g,
// so all KS offsets are lane values.
template <int C, int W>
struct Frag {
  static constexpr int TW = W + 2, NQ = C / 8, KS = Geo<C>::KS;
  static constexpr int NB = (C >= 32) ? 3 * (C / 32) : KS;
  int o[NB];
  __device__ __forceinline__ void init(int g, int lx) {
    if constexpr (C >= 32) {
#pragma unroll
      for (int kx = 0; kx < 3; ++kx)
#pragma unroll
        for (int cb = 0; cb < C / 32; ++cb) o[kx * (C / 32) + cb] = toff<C>(0, lx + kx, 4 * cb + g, TW);
    } else {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        int tap = (32 * ks + 8 * g) / C;
        if (tap > 8) tap = 8;  // C=16 tail k-step: A is zero there
        o[ks] = toff<C>(tap / 3, lx + tap % 3, (32 * ks + 8 * g) % C / 8, TW);
      }
    }
  }
  template <int ks>
  static constexpr int slot() {
    if constexpr (C >= 32) return ((32 * ks / C) % 3) * (C / 32) + (32 * ks % C) / 32;
    else return ks;
  }
  template <int ks, int pt>
  static constexpr int imm() {
    if constexpr (C >= 32) return ((32 * ks / C) / 3) * TW * NQ * 16 + pt * 16 * NQ * 16;
    else return pt * 16 * NQ * 16;
  }
};

template <int C, int W, int ks>
__device__ __forceinline__ void conv_issue(const unsigned (&ra)[Frag<C, W>::NB], bf16x8 (&B)[W / 16]) {
  if constexpr (W / 16 >= 1) B[0] = ds_read128<Frag<C, W>::template imm<ks, 0>()>(ra[Frag<C, W>::template slot<ks>()]);
  if constexpr (W / 16 >= 2) B[1] = ds_read128<Frag<C, W>::template imm<ks, 1>()>(ra[Frag<C, W>::template slot<ks>()]);
  static_assert(W / 16 <= 2, "conv_issue handles up to two pixel tiles");
}

// one k-step of the software pipeline: B of step ks lives in buffer ks%3;
// the reads of step ks+1 are in flight, those of ks+2 are issued after the
// MFMAs of ks (three buffers: a read never targets registers an MFMA issued
// in the previous step may still be reading).
template <int C, int W, int ks, typename Hook>
__device__ __forceinline__ void conv_step(const unsigned (&ra)[Frag<C, W>::NB],
                                          const bf16x8 (&A)[Geo<C>::OTW][Geo<C>::KS],
                                          f32x4 (&acc)[Geo<C>::OTW][W / 16], bf16x8 (&B)[3][W / 16], Hook& hook) {
  using G = Geo<C>;
  constexpr int PT = W / 16, KS = G::KS;
  if constexpr (ks < KS) {
    lgkm_wait<(ks + 1 < KS) ? PT : 0>();
#pragma unroll
    for (int pt = 0; pt < PT; ++pt)
#pragma unroll
      for (int t = 0; t < G::OTW; ++t)
        acc[t][pt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[t][ks], B[ks % 3][pt], acc[t][pt], 0, 0, 0);
    if constexpr (ks + 2 < KS) conv_issue<C, W, ks + 2>(ra, B[(ks + 2) % 3]);
    hook();
    conv_step<C, W, ks + 1>(ra, A, acc, B, hook);
  }
}

// conv GEMM of one output row (tile row r is the row above it), accumulated
// onto the caller's initial acc (the bias in the forward)
struct NoStepHook {
  __device__ __forceinline__ void operator()() const {}
};

// hook() runs once per k-step, after that step's MFMAs are issued (the
// backward interleaves its next-band DMA issue with the dgrad MFMAs that way)
template <int C, int W, typename Hook = NoStepHook>
__device__ __forceinline__ void conv_row(const unsigned char* tile, int r, const bf16x8 (&A)[Geo<C>::OTW][Geo<C>::KS],
                                         const Frag<C, W>& f, f32x4 (&acc)[Geo<C>::OTW][W / 16], Hook hook = {}) {
  using G = Geo<C>;
  constexpr int TW = W + 2, PT = W / 16;
  const unsigned rb = lds_u32(tile + r * TW * G::NQ * 16);
  unsigned ra[Frag<C, W>::NB];
#pragma unroll
  for (int k = 0; k < Frag<C, W>::NB; ++k) ra[k] = rb + (unsigned)f.o[k];
  bf16x8 B[3][PT];
  lgkm_wait<0>();  // nothing else of ours outstanding on the LDS counter
  conv_issue<C, W, 0>(ra, B[0]);
  if constexpr (G::KS > 1) conv_issue<C, W, 1>(ra, B[1]);
  conv_step<C, W, 0>(ra, A, acc, B, hook);
}

// ---------------------------------------------------------------------------
// Band conv (C >= 32): one wave = one 16-channel output tile over RB output
// rows.  The B fragment of input row ir (tap column kx, channel block cb)
// serves the MFMAs of every (output row r, tap row ky) with r + ky = ir, so
// RB+2 fragment reads feed 3*RB MFMAs per pixel tile (0.5 reads per MFMA
// at one o-tile per wave, the W fragments of that tile, 4*KS VGPRs, stay
// resident).  Fully unrolled, LDS reads software-pipelined two stages ahead.
// ---------------------------------------------------------------------------
template <int C, int W, int RB>
struct Band {
  static constexpr int TW = W + 2, NQ = C / 8, PT = W / 16, NCB = C / 32, KS = Geo<C>::KS;
  static constexpr int NR = RB + 2;             // input rows per band
  static constexpr int NS = 3 * NCB * NR;       // pipeline stages (kx, cb, input row)
  static constexpr int ROWB = TW * NQ * 16;     // LDS bytes per tile row
  static constexpr int PTB = 16 * NQ * 16;      // LDS bytes per 16-pixel tile
  static_assert(C % 32 == 0, "band conv needs whole 32-channel k-steps per tap");
  static_assert(NR * ROWB < 65536, "ds_read immediate offset range");
};

// input rows 0, 1 (the halo rows shared with the previous band) at baseh, rows 2.. at base
// (the same tile when baseh == base)
template <int C, int W, int RB, int S>
__device__ __forceinline__ void band_issue(unsigned base, unsigned baseh, const unsigned (&lo)[3 * Band<C, W, RB>::NCB],
                                           bf16x8 (&B)[Band<C, W, RB>::PT]) {
  using BD = Band<C, W, RB>;
  constexpr int blk = S / BD::NR, ir = S % BD::NR;
  const unsigned b = (ir < 2 ? baseh : base) + lo[blk];
  B[0] = ds_read128<ir * BD::ROWB>(b);
  if constexpr (BD::PT >= 2) B[1] = ds_read128<ir * BD::ROWB + BD::PTB>(b);
  static_assert(BD::PT <= 2, "band conv handles up to two pixel tiles");
}

// MFMAs of output row ir - KY (if inside the band) with tap (KY, kx)
template <int C, int W, int RB, int ir, int kx, int cb, int KY>
__device__ __forceinline__ void band_mfma(const bf16x8 (&A)[Geo<C>::KS], f32x4 (&acc)[RB][W / 16],
                                          const bf16x8 (&B)[W / 16]) {
  constexpr int r = ir - KY;
  if constexpr (r >= 0 && r < RB) {
    constexpr int ks = (KY * 3 + kx) * Band<C, W, RB>::NCB + cb;
#pragma unroll
    for (int pt = 0; pt < W / 16; ++pt)
      acc[r][pt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[ks], B[pt], acc[r][pt], 0, 0, 0);
  }
}

struct NoHook {
  template <typename U>
  __device__ __forceinline__ void operator()(U) const {}
};

// hook(integral_constant<int, u>) is called once for u = 0 .. NU-1, spread
// evenly over the pipeline stages (the forward interleaves the previous
// band's epilogue with this band's MFMAs that way)
template <int C, int W, int RB, int NU, int S, typename Hook>
__device__ __forceinline__ void band_step(unsigned base, unsigned baseh, const unsigned (&lo)[3 * Band<C, W, RB>::NCB],
                                          const bf16x8 (&A)[Geo<C>::KS], f32x4 (&acc)[RB][W / 16],
                                          bf16x8 (&B)[3][W / 16], Hook& hook) {
  using BD = Band<C, W, RB>;
  constexpr int PT = BD::PT;
  if constexpr (S < BD::NS) {
    constexpr int blk = S / BD::NR, ir = S % BD::NR;
    constexpr int kx = blk / BD::NCB, cb = blk % BD::NCB;
    lgkm_wait<(S + 1 < BD::NS) ? PT : 0>();
    band_mfma<C, W, RB, ir, kx, cb, 0>(A, acc, B[S % 3]);
    band_mfma<C, W, RB, ir, kx, cb, 1>(A, acc, B[S % 3]);
    band_mfma<C, W, RB, ir, kx, cb, 2>(A, acc, B[S % 3]);
    if constexpr (S + 2 < BD::NS) band_issue<C, W, RB, S + 2>(base, baseh, lo, B[(S + 2) % 3]);
    if constexpr (NU > 0) {
      constexpr int SP = BD::NS / NU;
      if constexpr (SP > 0 && S % SP == SP / 2 && S / SP < NU) hook(std::integral_constant<int, S / SP>{});
    }
    band_step<C, W, RB, NU, S + 1>(base, baseh, lo, A, acc, B, hook);
  }
}

// acc[r][pt] += conv over the RB output rows whose first input row is the
// tile row at LDS byte address `base`
template <int C, int W, int RB, int NU = 0, typename Hook = NoHook>
__device__ __forceinline__ void conv_band2(unsigned base, unsigned baseh, const unsigned (&lo)[3 * Band<C, W, RB>::NCB],
                                           const bf16x8 (&A)[Geo<C>::KS], f32x4 (&acc)[RB][W / 16], Hook hook = {}) {
  bf16x8 B[3][W / 16];
  lgkm_wait<0>();
  band_issue<C, W, RB, 0>(base, baseh, lo, B[0]);
  band_issue<C, W, RB, 1>(base, baseh, lo, B[1]);
  band_step<C, W, RB, NU, 0>(base, baseh, lo, A, acc, B, hook);
}
template <int C, int W, int RB, int NU = 0, typename Hook = NoHook>
__device__ __forceinline__ void conv_band(unsigned base, const unsigned (&lo)[3 * Band<C, W, RB>::NCB],
                                          const bf16x8 (&A)[Geo<C>::KS], f32x4 (&acc)[RB][W / 16], Hook hook = {}) {
  conv_band2<C, W, RB, NU, Hook>(base, base, lo, A, acc, hook);
}

template <int C, int W, int RB>
__device__ __forceinline__ void band_lane_offsets(int g, int lx, unsigned (&lo)[3 * Band<C, W, RB>::NCB]) {
  using BD = Band<C, W, RB>;
#pragma unroll
  for (int kx = 0; kx < 3; ++kx)
#pragma unroll
    for (int cb = 0; cb < BD::NCB; ++cb) lo[kx * BD::NCB + cb] = (unsigned)toff<C>(0, lx + kx, 4 * cb + g, BD::TW);
}

// W^T fragments of one 16-channel output tile
template <int C>
__device__ __forceinline__ void load_A1(const bf16* __restrict__ wpack, int ot, int lane, bf16x8 (&A)[Geo<C>::KS]) {
#pragma unroll
  for (int ks = 0; ks < Geo<C>::KS; ++ks)
    A[ks] = *(const bf16x8*)(wpack + (((long)ot * Geo<C>::KS + ks) * 64 + lane) * 8);
}

// load_A1 / the 4 bias values of lane group g by untracked loads (see
// gload128_untracked): for the stacks' per-block reloads, whose results the
// next item's barrier_vm retires.  Unconditional loads into the registers the
// values live in (a null bias reads the zero page): a conditional load would
// make hipcc merge the two values with copies that read the registers before
// the load retires.
template <int C, int KS0 = 0>
__device__ __forceinline__ void load_A1_untracked_at(const unsigned char* base, unsigned voff, bf16x8 (&A)[Geo<C>::KS]) {
  if constexpr (KS0 < Geo<C>::KS) {
    u32x4 v = __builtin_bit_cast(u32x4, A[KS0]);
    // the base advances by 4 KiB every 4 loads (an SALU add): only a load right after
    // such an add (or the readfirstlane of the first) needs the 5 wait states
    gload128_untracked<(KS0 % 4) * 1024, KS0 % 4 == 0>(v, base + (KS0 / 4) * 4096, voff);
    A[KS0] = __builtin_bit_cast(bf16x8, v);
    load_A1_untracked_at<C, KS0 + 1>(base, voff, A);
  }
}
template <int C>
__device__ __forceinline__ void load_A1_untracked(const bf16* __restrict__ wpack, int ot, int lane,
                                                  bf16x8 (&A)[Geo<C>::KS]) {
  const auto* base = (const unsigned char*)uniform_ptr((const unsigned char*)wpack + (long)ot * Geo<C>::KS * 1024);
  load_A1_untracked_at<C>(base, (unsigned)lane * 16u, A);
}
// b: the wave's 16 bias values (wave-uniform); lane group g reads 4 of them
__device__ __forceinline__ void load_bias4_untracked(const float* __restrict__ b, int g, float (&bz)[4]) {
  const void* base = uniform_ptr(b ? (const void*)b : (const void*)g_zero_page);
  const unsigned voff = (unsigned)g * 16u;
  gload32_untracked<0>(bz[0], base, voff);
  gload32_untracked<4>(bz[1], base, voff);
  gload32_untracked<8>(bz[2], base, voff);
  gload32_untracked<12>(bz[3], base, voff);
}

template <int C>
__device__ __forceinline__ void load_A(const bf16* __restrict__ wpack, int oh, int lane,
                                       bf16x8 (&A)[Geo<C>::OTW][Geo<C>::KS]) {
  using G = Geo<C>;
#pragma unroll
  for (int t = 0; t < G::OTW; ++t)
#pragma unroll
    for (int ks = 0; ks < G::KS; ++ks)
      A[t][ks] = *(const bf16x8*)(wpack + (((long)(oh * G::OTW + t) * G::KS + ks) * 64 + lane) * 8);
}

// contiguous run of items for this workgroup
__device__ __forceinline__ void item_range(int items, int* i0, int* i1) {
  const int per = items / (int)gridDim.x, rem = items % (int)gridDim.x;
  const int b = blockIdx.x;
  *i0 = b * per + min(b, rem);
  *i1 = *i0 + per + (b < rem ? 1 : 0);
}

// (image, band) of consecutive items without a division per item
struct ItemCursor {
  int n, b;
  __device__ __forceinline__ ItemCursor(int it, int nb) : n(it / nb), b(it % nb) {}
  __device__ __forceinline__ void next(int nb) {
    if (++b == nb) {
      b = 0;
      ++n;
    }
  }
};

// ===========================================================================
// forward
// ===========================================================================
template <int C, int W, int BR, int MODE, int NW>
__global__ __launch_bounds__(64 * NW) void k_fwd(const bf16* __restrict__ x, const bf16* __restrict__ resid,
                                             bf16* __restrict__ y, uint8_t* __restrict__ mask,
                                             const bf16* __restrict__ wpack, const float* __restrict__ bias,
                                             float h, int N, int H) {
  using G = Geo<C>;
  constexpr int TW = W + 2, PT = W / 16, NQ = G::NQ, OTW = G::OTW;
  constexpr int TILE = (BR + 2) * TW * NQ * 16;
  constexpr int RS = NW / G::OSPLIT;  // waves splitting the band's rows
  constexpr bool EULER = MODE == FWD_EULER;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int oh = wave % G::OSPLIT, rg = wave / G::OSPLIT;
  const int g = lane >> 4, lx = lane & 15;

  bf16x8 A[OTW][G::KS];
  load_A<C>(wpack, oh, lane, A);
  Frag<C, W> boff;
  boff.init(g, lx);
  float bz[OTW][4];
#pragma unroll
  for (int t = 0; t < OTW; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) bz[t][e] = bias ? bias[16 * (oh * OTW + t) + 4 * g + e] : 0.f;

  zero_halo_cols<C, W>(lds, BR + 2, tid, 64 * NW);
  zero_halo_cols<C, W>(lds + TILE, BR + 2, tid, 64 * NW);
  const int nb = (H + BR - 1) / BR;
  int i0, i1;
  item_range(N * nb, &i0, &i1);
  ItemCursor cur(i0, nb), nxt(i0, nb);
  if (i0 < i1) {
    const int y0 = cur.b * BR;
    dma_rows<C, W>(x, lds, cur.n, y0 - 1, min(BR, H - y0) + 2, H, wave, NW, lane);
  }
  nxt.next(nb);
  int nst = 0;  // global stores this wave issued after the DMA it must now wait for
  for (int it = i0; it < i1; ++it, cur.next(nb), nxt.next(nb)) {
    const int buf = (it - i0) & 1;
    unsigned char* tile = lds + buf * TILE;
    barrier_vm(nst);  // this item's DMA has landed; the other buffer is free
    nst = 0;
    if (it + 1 < i1) {
      const int y1 = nxt.b * BR;
      dma_rows<C, W>(x, lds + (buf ^ 1) * TILE, nxt.n, y1 - 1, min(BR, H - y1) + 2, H, wave, NW, lane);
    }
    const int n = cur.n, y0 = cur.b * BR;
    const int rows = min(BR, H - y0);
    for (int r = rg; r < rows; r += RS) {
      f32x4 acc[OTW][PT];
#pragma unroll
      for (int t = 0; t < OTW; ++t)
#pragma unroll
        for (int pt = 0; pt < PT; ++pt) acc[t][pt] = f32x4{bz[t][0], bz[t][1], bz[t][2], bz[t][3]};
      conv_row<C, W>(tile, r, A, boff, acc);
      const int gy = y0 + r;
      nst += PT * (OTW + ((EULER && mask) ? 1 : 0));
#pragma unroll
      for (int pt = 0; pt < PT; ++pt) {
        const int px = 16 * pt + lx;
        unsigned mword = 0;
#pragma unroll
        for (int t = 0; t < OTW; ++t) {
          const int o0 = 16 * (oh * OTW + t) + 4 * g;
          bf16x4 o4;
          if constexpr (EULER) {
            // residual: x itself (LDS tile) or, for the second RK2 stage, the step's input
            const bf16x4 xr = resid ? *(const bf16x4*)(resid + (((long)n * H + gy) * W + px) * C + o0)
                                    : *(const bf16x4*)(tile + toff<C>(r + 1, px + 1, o0 >> 3, TW) + (o0 & 4) * 2);
            unsigned nib = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float z = acc[t][pt][e];
              const bool pos = z > 0.f;  // relu'(z) as TF's ReluGrad: z > 0
              nib |= (pos ? 1u : 0u) << e;
              o4[e] = (bf16)fmaf(h, pos ? z : 0.f, (float)xr[e]);
            }
            mword |= nib << (16 * t + 4 * g);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) o4[e] = (bf16)acc[t][pt][e];
          }
          *(bf16x4*)(y + (((long)n * H + gy) * W + px) * C + o0) = o4;
        }
        if constexpr (EULER) {
          // OR over the four lane groups g (lanes lx, lx+16, lx+32, lx+48)
          const auto s16 = __builtin_amdgcn_permlane16_swap(mword, mword, false, false);
          mword = s16[0] | s16[1];
          const auto s32 = __builtin_amdgcn_permlane32_swap(mword, mword, false, false);
          mword = s32[0] | s32[1];
          if (mask && g == 0) {
            uint8_t* mp = mask + ((((long)n * H + gy) * W + px) * C + 16 * oh * OTW) / 8;
            if constexpr (OTW == 2)
              *(uint32_t*)mp = mword;
            else
              *(uint16_t*)mp = (uint16_t)mword;
          }
        }
      }
    }
  }
}

template <int NU, int U = 0, typename F, typename Acc, typename Xr, typename Cur>
__device__ __forceinline__ void epi_all_units(F& f, const Acc& acc, const Xr& xr, const Cur& c) {
  if constexpr (U < NU) {
    f(std::integral_constant<int, U>{}, acc, xr, c);
    epi_all_units<NU, U + 1>(f, acc, xr, c);
  }
}

// Forward, band form with a software pipeline across bands: the MFMAs of
// band i+1 are interleaved with the epilogue (VALU + stores) of band i, so
// the matrix pipe and the vector ALU of one wave work at the same time.
// RESG (second RK2 stage, default): the residual `resid` read from global
// memory.  Band i+1's loads are issued right after band i+2's DMA and
// consumed (an empty asm that reads them) right after the next barrier, before
// any later DMA: hipcc's own vmcnt wait for a load counts only the memory ops
// it sees, so a use behind a younger inline-asm DMA would wait for that DMA.
template <int C, int W, int BR, int MODE, int NW, bool RESG = false>
__global__ __launch_bounds__(64 * NW, 2) void k_fwd_pipe(const bf16* __restrict__ x, const bf16* __restrict__ resid,
                                                  bf16* __restrict__ y, uint8_t* __restrict__ mask,
                                                  const bf16* __restrict__ wpack, const float* __restrict__ bias,
                                                  float h, int N, int H) {
  using G = Geo<C>;
  constexpr int TW = W + 2, PT = W / 16, NQ = G::NQ, OT = C / 16;
  constexpr int TILE = (BR + 2) * TW * NQ * 16;
  static_assert(NW % OT == 0, "waves must cover the o-tiles");
  constexpr int RS = NW / OT, RB = BR / RS;
  static_assert(BR % RS == 0, "row groups must split the band");
  using BD = Band<C, W, RB>;
  // epilogue units: (row, pixel tile), or rows with both pixel tiles stored
  // as 16-B chunks
  constexpr bool ST16 = PT == 2;
  constexpr int NU = ST16 ? RB : RB * PT;
  constexpr bool EULER = MODE == FWD_EULER;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ot = wave % OT, rg = wave / OT;
  const int g = lane >> 4, lx = lane & 15;
  const int o0 = 16 * ot + 4 * g;
  const int r0 = rg * RB;

  bf16x8 A[G::KS];
  load_A1<C>(wpack, ot, lane, A);
  unsigned lo[3 * BD::NCB];
  band_lane_offsets<C, W, RB>(g, lx, lo);
  float bz[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) bz[e] = bias ? bias[o0 + e] : 0.f;
  const unsigned ly = (unsigned)(lx * C + o0);
  const unsigned lm = (unsigned)(lx * (C / 8) + 2 * ot);
  const unsigned lxr = (unsigned)(toff<C>(r0 + 1, lx + 1, o0 >> 3, TW) + (o0 & 4) * 2);

  zero_halo_cols<C, W>(lds, BR + 2, tid, 64 * NW);
  zero_halo_cols<C, W>(lds + TILE, BR + 2, tid, 64 * NW);
  const int nb = (H + BR - 1) / BR;
  int i0, i1;
  item_range(N * nb, &i0, &i1);
  if (i0 >= i1) return;
  ItemCursor cur(i0, nb), nx1(i0, nb), nx2(i0, nb);  // items it, it+1, it+2
  nx1.next(nb);
  nx2.next(nb);
  nx2.next(nb);
  auto dma = [&](const ItemCursor& c, int buf) {
    const int yy = c.b * BR;
    dma_rows<C, W>(x, lds + buf * TILE, c.n, yy - 1, min(BR, H - yy) + 2, H, wave, NW, lane);
  };
  // band c continues band p's image (p's tile in the other buffer, complete):
  // its halo rows 0, 1 are p's rows BR, BR+1 -> copy them (interior columns),
  // DMA only rows 2..
  auto dma_next2 = [&](const ItemCursor& c, const ItemCursor& p, int buf) {
    if (c.n != p.n || c.b != p.b + 1) {
      dma(c, buf);
      return;
    }
    const int yy = c.b * BR;
    constexpr int ROWB = TW * NQ * 16;
    dma_rows<C, W>(x, lds + buf * TILE + 2 * ROWB, c.n, yy + 1, min(BR, H - yy), H, wave, NW, lane);
    // plain LDS accesses (the DMA is inline asm, invisible to the compiler,
    // so it waits only lgkmcnt for these; asm reads with a deferred wait are
    // unsafe where hipcc copies their results before the wait)
    const uint4* src = (const uint4*)(lds + (buf ^ 1) * TILE + BR * ROWB);
    uint4* dst = (uint4*)(lds + buf * TILE);
    constexpr int NCH = 2 * W * NQ;
    for (int i = tid; i < NCH; i += 64 * NW) dst[((i / (W * NQ)) * TW + 1) * NQ + i % (W * NQ)] =
        src[((i / (W * NQ)) * TW + 1) * NQ + i % (W * NQ)];
  };
  int nst = 0;  // vector-memory ops this wave issued after the DMA the next barrier waits for
  // residual of a band: x from its LDS tile (read after the band's conv)
  auto xres_read = [&](int buf, u32x2 (&xr)[RB][PT]) {
    if constexpr (EULER && !RESG) {
      const unsigned tb = lds_u32(lds + buf * TILE) + lxr;
#pragma unroll
      for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int pt = 0; pt < PT; ++pt) xr[r][pt] = lds_rd64(tb + (unsigned)(r * BD::ROWB + pt * BD::PTB));
      lgkm_wait<0>();
    }
  };
  // RESG: every lane issues exactly RB*PT loads (rows past the image end
  // re-read its last row), so the barrier counts stay exact
  const unsigned lres = (unsigned)(2 * (lx * C + o0));
  auto xg_load = [&](const ItemCursor& c, u32x2 (&xr)[RB][PT]) {
    if constexpr (RESG) {
      const int y0 = c.b * BR, rows = min(BR, H - y0);
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const int ur = __builtin_amdgcn_readfirstlane((c.n * H + y0 + min(r0 + r, rows - 1)) * W);
        const unsigned char* rb = (const unsigned char*)(resid + (long)ur * C);
#pragma unroll
        for (int pt = 0; pt < PT; ++pt) xr[r][pt] = *(const u32x2*)(rb + lres + (unsigned)(2 * 16 * pt * C));
      }
      nst += RB * PT;
    }
  };
  auto xg_consume = [&](u32x2 (&xr)[RB][PT]) {
    if constexpr (RESG) {
#pragma unroll
      for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int pt = 0; pt < PT; ++pt) asm volatile("" : "+v"(xr[r][pt]));
    }
  };
  auto init = [&](f32x4 (&acc)[RB][PT]) {
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int pt = 0; pt < PT; ++pt) acc[r][pt] = f32x4{bz[0], bz[1], bz[2], bz[3]};
  };
  // y and the relu-mask word of output row r, pixel tile pt (every lane
  // ends with the 16-bit mask word of its pixel: OR over the 4 lane rows)
  auto epi_vals = [&](int r, int pt, const f32x4 (&acc)[RB][PT], const u32x2 (&xr)[RB][PT], u32x2& ov,
                      unsigned& mword) {
    bf16x4 o4;
    mword = 0;
    if constexpr (EULER) {
      const bf16x4 xv = *(const bf16x4*)&xr[r][pt];
      unsigned nib = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float z = acc[r][pt][e];
        const bool pos = z > 0.f;  // relu'(z) as TF's ReluGrad: z > 0
        nib |= (pos ? 1u : 0u) << e;
        const float rz = __builtin_bit_cast(float, __builtin_bit_cast(unsigned, z) & (pos ? ~0u : 0u));
        o4[e] = (bf16)fmaf(h, rz, (float)xv[e]);
      }
      mword = nib << (4 * g);
      const auto s16 = __builtin_amdgcn_permlane16_swap(mword, mword, false, false);
      mword = s16[0] | s16[1];
      const auto s32 = __builtin_amdgcn_permlane32_swap(mword, mword, false, false);
      mword = s32[0] | s32[1];
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) o4[e] = (bf16)acc[r][pt][e];
    }
    ov = *(const u32x2*)&o4;
  };
  // one epilogue unit of the band at cursor c
  auto epi_unit = [&](auto U, const f32x4 (&acc)[RB][PT], const u32x2 (&xr)[RB][PT], const ItemCursor& c) {
    constexpr int u = decltype(U)::value;
    const int y0 = c.b * BR;
    if constexpr (ST16) {
      // row r, both pixel tiles: a 16-lane row swap between the tiles gives
      // lane row g the 8 channels 16*ot + 8*(g>>1) of pixel 16*(g&1) + lx
      constexpr int r = u;
      if (r0 + r >= min(BR, H - y0)) return;
      const long row = ((long)c.n * H + y0 + r0 + r) * W;
      nst += (EULER && mask) ? 2 : 1;
      u32x2 ov[2];
      unsigned mw[2];
      epi_vals(r, 0, acc, xr, ov[0], mw[0]);
      epi_vals(r, 1, acc, xr, ov[1], mw[1]);
      const auto s0 = __builtin_amdgcn_permlane16_swap(ov[0][0], ov[1][0], false, false);
      const auto s1 = __builtin_amdgcn_permlane16_swap(ov[0][1], ov[1][1], false, false);
      *(u32x4*)(y + (row + 16 * (g & 1) + lx) * C + 16 * ot + 8 * (g >> 1)) = u32x4{s0[0], s1[0], s0[1], s1[1]};
      if (EULER && mask && g < 2) *(uint16_t*)(mask + (row + 16 * g) * (C / 8) + lm) = (uint16_t)(g ? mw[1] : mw[0]);
    } else {
      constexpr int r = u / PT, pt = u % PT;
      if (r0 + r >= min(BR, H - y0)) return;
      const long row = ((long)c.n * H + y0 + r0 + r) * W + 16 * pt;
      nst += (EULER && mask) ? 2 : 1;
      u32x2 ov;
      unsigned mword;
      epi_vals(r, pt, acc, xr, ov, mword);
      if (EULER && mask && g == 0) *(uint16_t*)(mask + row * (C / 8) + lm) = (uint16_t)mword;
      *(u32x2*)(y + row * C + ly) = ov;
    }
  };
  auto epi_all = [&](const f32x4 (&acc)[RB][PT], const u32x2 (&xr)[RB][PT], const ItemCursor& c) {
    epi_all_units<NU>(epi_unit, acc, xr, c);
  };

  f32x4 accA[RB][PT], accB[RB][PT];
  u32x2 xrA[RB][PT], xrB[RB][PT];
  // prologue: band i0 computed (its epilogue waits for the next band's MFMAs)
  dma(cur, 0);
  barrier_vm(0);
  if (i0 + 1 < i1) dma(nx1, 1);
  xg_load(cur, xrA);
  init(accA);
  conv_band<C, W, RB>(lds_u32(lds + r0 * BD::ROWB), lo, A, accA);
  xres_read(0, xrA);
  int it = i0;
  while (true) {
    // accA / xrA: band it.  In flight: DMA of band it+1 into buffer (it+1-i0)&1.
    if (it + 1 >= i1) {
      epi_all(accA, xrA, cur);
      break;
    }
    ASR_STAMP(it - i0, 0);
    barrier_vm(nst);  // band it+1 landed, every wave is done with band it's tile
    ASR_STAMP(it - i0, 1);
    nst = 0;
    xg_consume(xrA);
    if (it + 2 < i1) dma_next2(nx2, nx1, (it - i0) & 1);
    xg_load(nx1, xrB);
    ASR_STAMP(it - i0, 2);
    init(accB);
    {
      const ItemCursor c = cur;
      auto hook = [&](auto U) { epi_unit(U, accA, xrA, c); };
      conv_band<C, W, RB, NU>(lds_u32(lds + ((it + 1 - i0) & 1) * TILE + r0 * BD::ROWB), lo, A, accB, hook);
    }
    ASR_STAMP(it - i0, 3);
    xres_read((it + 1 - i0) & 1, xrB);
    ASR_STAMP(it - i0, 4);
    ++it;
    cur.next(nb);
    nx1.next(nb);
    nx2.next(nb);
    // the same with the roles of A and B swapped
    if (it + 1 >= i1) {
      epi_all(accB, xrB, cur);
      break;
    }
    ASR_STAMP(it - i0, 0);
    barrier_vm(nst);
    ASR_STAMP(it - i0, 1);
    nst = 0;
    xg_consume(xrB);
    if (it + 2 < i1) dma_next2(nx2, nx1, (it - i0) & 1);
    xg_load(nx1, xrA);
    ASR_STAMP(it - i0, 2);
    init(accA);
    {
      const ItemCursor c = cur;
      auto hook = [&](auto U) { epi_unit(U, accB, xrB, c); };
      conv_band<C, W, RB, NU>(lds_u32(lds + ((it + 1 - i0) & 1) * TILE + r0 * BD::ROWB), lo, A, accA, hook);
    }
    ASR_STAMP(it - i0, 3);
    xres_read((it + 1 - i0) & 1, xrA);
    ASR_STAMP(it - i0, 4);
    ++it;
    cur.next(nb);
    nx1.next(nb);
    nx2.next(nb);
  }
}

// Forward, band form at three waves per SIMD (C = 64; 3 WGs of 4 waves per
// CU, <= 168 VGPRs): no cross-band software pipeline.  Each wave runs its
// o-tile's band conv, then the band's epilogue; the other two workgroups on
// the CU keep the matrix pipe busy meanwhile.  The epilogue works on the
// regrouped accumulators (v_permlane16_swap: lane (lx, g) owns channels
// 16*ot + 8*(g>>1) + 0..7 of pixel lx + 16*(g&1)): the residual is one
// ds_read_b128 of the band's LDS tile, y one 16-B store, the relu bits one
// byte per lane (v_med3 + v_lshl_or, relu as an integer max on the bit
// pattern).  MFMA accumulation order and rounding equal k_fwd_pipe's, so both
// kernels give bitwise the same y and mask.
// RESG (second RK2 stage): the residual is `resid` (the step input), not the
// conv input x: 16-B global loads in the regrouped layout, issued before the conv.
template <int C, int W, int BR, int MODE, int WPE, bool RESG = false>
__global__ __launch_bounds__(256, WPE) void k_fwd3(const bf16* __restrict__ x, const bf16* __restrict__ resid,
                                                   bf16* __restrict__ y, uint8_t* __restrict__ mask,
                                                   const bf16* __restrict__ wpack, const float* __restrict__ bias,
                                                   float h, int N, int H) {
  using G = Geo<C>;
  constexpr int TW = W + 2, NQ = G::NQ, OT = C / 16, NW = 4, RB = BR;
  static_assert(OT == NW && W == 32, "one 16-channel o-tile per wave, two pixel tiles");
  using BD = Band<C, W, RB>;
  constexpr int TILE = (BR + 2) * BD::ROWB;
  constexpr bool EULER = MODE == FWD_EULER;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ot = wave, g = lane >> 4, lx = lane & 15;
  const int o0 = 16 * ot + 4 * g;
  const int px = lx + 16 * (g & 1), cg = 2 * ot + (g >> 1);  // after the regroup: pixel, 16-B channel chunk

  bf16x8 A[G::KS];
  load_A1<C>(wpack, ot, lane, A);
  unsigned lo[3 * BD::NCB];
  band_lane_offsets<C, W, RB>(g, lx, lo);
  float bz[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) bz[e] = bias ? bias[o0 + e] : 0.f;
  const unsigned lxr = (unsigned)toff<C>(1, px + 1, cg, TW);  // output row 0's residual chunk
  const unsigned ly = (unsigned)(px * C + 8 * cg) * 2u, lm = (unsigned)(px * (C / 8) + cg);

  zero_halo_cols<C, W>(lds, BR + 2, tid, 64 * NW);
  zero_halo_cols<C, W>(lds + TILE, BR + 2, tid, 64 * NW);
  const int nb = (H + BR - 1) / BR;
  int i0, i1;
  item_range(N * nb, &i0, &i1);
  if (i0 >= i1) return;
  ItemCursor cur(i0, nb), nxt(i0, nb);
  nxt.next(nb);
  {
    const int yy = cur.b * BR;
    dma_rows<C, W>(x, lds, cur.n, yy - 1, min(BR, H - yy) + 2, H, wave, NW, lane);
  }
  int nst = 0;  // vector-memory ops issued after the DMA the next barrier waits for
  ASR_BCLK(0, 0);
  for (int it = i0; it < i1; ++it, cur.next(nb), nxt.next(nb)) {
    const int buf = (it - i0) & 1;
    if (wave == 0) ASR_BTR(0, 0, it - i0, 0);
    barrier_vm_usual<2 * BR>(nst);  // band it landed; every wave is done with band it-1's tile
    if (wave == 0) ASR_BTR(0, 0, it - i0, 1);
    nst = 0;
    if (it + 1 < i1) {
      // the next band into the other buffer; its rows 0, 1 are this band's rows
      // BR, BR+1 when it continues the image (copied inside LDS, the rest by DMA)
      unsigned char* nt = lds + (buf ^ 1) * TILE;
      const int yy = nxt.b * BR;
      if (nxt.n == cur.n && nxt.b == cur.b + 1) {
        dma_rows<C, W>(x, nt + 2 * BD::ROWB, nxt.n, yy + 1, min(BR, H - yy), H, wave, NW, lane);
        const uint4* src = (const uint4*)(lds + buf * TILE + BR * BD::ROWB);
        uint4* dst = (uint4*)nt;
        constexpr int NCH = 2 * W * NQ;
        for (int i = tid; i < NCH; i += 64 * NW) {
          const int o = ((i / (W * NQ)) * TW + 1) * NQ + i % (W * NQ);
          dst[o] = src[o];
        }
      } else {
        dma_rows<C, W>(x, nt, nxt.n, yy - 1, min(BR, H - yy) + 2, H, wave, NW, lane);
      }
    }
    const unsigned tb = lds_u32(lds + buf * TILE);
    u32x4 xr[RB];
    if constexpr (RESG) {  // rows past the image end re-read its last row (never stored)
      const int y0 = cur.b * BR, rows = min(BR, H - y0);
      const unsigned char* rb = (const unsigned char*)(resid + ((long)cur.n * H + y0) * W * C) + ly;
#pragma unroll
      for (int r = 0; r < RB; ++r) xr[r] = *(const u32x4*)(rb + (long)min(r, rows - 1) * W * C * 2);
    }
    f32x4 acc[RB][2];
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int pt = 0; pt < 2; ++pt) acc[r][pt] = f32x4{bz[0], bz[1], bz[2], bz[3]};
    if (wave == 0) ASR_BTR(0, 0, it - i0, 2);
    conv_band<C, W, RB>(tb, lo, A, acc);
    if (wave == 0) ASR_BTR(0, 0, it - i0, 3);
    if constexpr (EULER && !RESG) {
#pragma unroll
      for (int r = 0; r < RB; ++r) xr[r] = lds_rd128(tb + lxr + (unsigned)(r * BD::ROWB));
      lgkm_wait<0>();
    }
    const int y0 = cur.b * BR, rows = min(BR, H - y0);
    const long rowb = ((long)cur.n * H + y0) * W;
    unsigned char* yb = (unsigned char*)(y + rowb * C) + ly;
    uint8_t* mb = mask ? mask + rowb * (C / 8) + lm : nullptr;
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      if (r >= rows) break;
      float z[8];
      regroup(acc[r][0], acc[r][1], z);
      u32x4 yw;
      if constexpr (EULER) {
        unsigned bits = 0;
        static_for<0, 4>([&](auto dc) {
          constexpr int d = decltype(dc)::value;
          const int ra = max(__float_as_int(z[2 * d]), 0), rb = max(__float_as_int(z[2 * d + 1]), 0);
          yw[d] = pk_bf16(fmaf(h, __int_as_float(ra), lo_f(xr[r][d])), fmaf(h, __int_as_float(rb), hi_f(xr[r][d])));
          bits = d == 0 ? bit01(ra) : lshl_or<2 * d>(bit01(ra), bits);
          bits = lshl_or<2 * d + 1>(bit01(rb), bits);
        });
        if (mb) {
          mb[r * W * (C / 8)] = (uint8_t)bits;
          ++nst;
        }
      } else {
#pragma unroll
        for (int d = 0; d < 4; ++d) yw[d] = pk_bf16(z[2 * d], z[2 * d + 1]);
      }
      *(u32x4*)(yb + r * W * C * 2) = yw;
      ++nst;
    }
    if (wave == 0) ASR_BTR(0, 0, it - i0, 4);
  }
  ASR_BCLK(0, 1);
}

// ===========================================================================
// Stack forward (C=64, W=32, BR=4, Euler): all L blocks of a network in ONE
// launch.  The images do not interact (3x3 SAME conv per image, no batch
// statistics), so a workgroup owns a contiguous run of whole images and walks
// (layer, image, band) items: block l+1 of an image reads only what this
// workgroup wrote for block l, and no workgroup ever waits for another.  The
// per-band protocol is k_fwd3's (band conv + regrouped epilogue, next band's
// rows by LDS-DMA into the other buffer, halo rows copied within an image).
// Replaces L launches of k_fwd3: no per-launch fill and drain, and no tail of
// workgroups with one band more than the rest (whole images per workgroup).
// Ordering: the DMA of item it+1 is issued after the barrier of item it, when
// every wave's stores of items <= it-1 have been waited for (barrier_vm counts
// only the previous item's stores as still in flight), so the first band of
// block l+1 (it reads rows -1..4 of block l's output, written by the first
// two bands of the image) needs >= 4 bands per workgroup and block: the host
// checks nb >= 4.  Training: activations are distinct buffers per block,
// written once in this launch.  Inference (slots = 2): x_{l+1} goes to slot
// l % 2 of ys, so block l+1 overwrites x_l; a workgroup finishes every item of
// block l (whole images, its own) before it writes block l+1, and its own
// stores and DMA reads meet in its CU's L1, so no line can be stale either.
// ===========================================================================
// RK2 (BASELINE config 5): 2L stages, stage 2l = the first (x_l -> xmid_l, h/2,
// mask1), stage 2l+1 the second (xmid_l -> x_{l+1}, h, mask2) with the residual
// x_l from global memory (16-B loads in the regrouped layout, as k_fwd3<..., RESG>).
template <int C, int W, int BR, bool RK2 = false>
__global__ __launch_bounds__(256, 2) void k_fwd3_stack(const bf16* __restrict__ x0, bf16* __restrict__ ys,
                                                       long y_stride, uint8_t* __restrict__ masks, long mask_stride,
                                                       const bf16* __restrict__ wpack, long w_stride,
                                                       const float* __restrict__ bias, long bias_stride, float h,
                                                       int N, int H, int L, int slots,
                                                       bf16* __restrict__ xm = nullptr,
                                                       uint8_t* __restrict__ masks2 = nullptr) {
  using G = Geo<C>;
  constexpr int TW = W + 2, NQ = G::NQ, OT = C / 16, NW = 4, RB = BR;
  static_assert(OT == NW && W == 32, "one 16-channel o-tile per wave, two pixel tiles");
  using BD = Band<C, W, RB>;
  constexpr int TILE = (BR + 2) * BD::ROWB;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ot = wave, g = lane >> 4, lx = lane & 15;
  const int o0 = 16 * ot + 4 * g;
  const int px = lx + 16 * (g & 1), cg = 2 * ot + (g >> 1);

  // whole images per workgroup
  const int n0 = (int)((long)blockIdx.x * N / gridDim.x), n1 = (int)((long)(blockIdx.x + 1) * N / gridDim.x);
  if (n0 >= n1) return;
  const int nb = (H + BR - 1) / BR, per = (n1 - n0) * nb;  // items per block
  // items walk stages (blocks, or RK2 half steps): block, input, output, mask, step of stage st
  auto blk_of = [&](int st) { return RK2 ? st >> 1 : st; };
  // slots: 0 = one buffer per block (training), 2 = ping-pong (inference; Euler only)
  auto slot_of = [&](int l) -> long { return slots > 0 ? (long)(l % slots) : (long)l; };
  auto xin_of = [&](int l) -> const bf16* { return l == 0 ? x0 : ys + slot_of(l - 1) * y_stride; };
  auto src_of = [&](int st) -> const bf16* {
    if constexpr (RK2) return (st & 1) ? xm + (long)(st >> 1) * y_stride : xin_of(st >> 1);
    else return xin_of(st);
  };
  auto out_of = [&](int st) -> bf16* {
    if constexpr (RK2) return ((st & 1) ? ys : xm) + (long)(st >> 1) * y_stride;
    else return ys + slot_of(st) * y_stride;
  };
  auto mask_of = [&](int st) -> uint8_t* {
    uint8_t* m = (RK2 && (st & 1)) ? masks2 : masks;
    return m ? m + (long)blk_of(st) * mask_stride : nullptr;
  };

  // A and the bias by untracked loads, here and at every block switch: the
  // next item's barrier_vm retires them (tracked, hipcc would wait vmcnt(0)
  // before each band's first MFMA, i.e. for the next band's DMA as well)
  bf16x8 A[G::KS] = {};
  load_A1_untracked<C>(wpack, ot, lane, A);
  unsigned lo[3 * BD::NCB];
  band_lane_offsets<C, W, RB>(g, lx, lo);
  float bz[4] = {0.f, 0.f, 0.f, 0.f};
  load_bias4_untracked(bias ? bias + 16 * ot : nullptr, g, bz);
  const unsigned lxr = (unsigned)toff<C>(1, px + 1, cg, TW);
  const unsigned ly = (unsigned)(px * C + 8 * cg) * 2u, lm = (unsigned)(px * (C / 8) + cg);

  // A ring of three tiles: a band that continues the previous band's image
  // reads its two halo rows where that band's tile holds them (rows BR, BR+1), so only its
  // BR new rows are DMA'd and nothing is copied inside LDS.  The DMA of band it+1 goes to
  // the tile band it-2 used, which band it-1 read last (as its halo rows): free after
  // band it's barrier.  (2 tiles: the halo rows copied into the next tile.)
  constexpr int NT = 3;
#pragma unroll
  for (int k = 0; k < NT; ++k) zero_halo_cols<C, W>(lds + k * TILE, BR + 2, tid, 64 * NW);
  constexpr int IPR = W / G::PPI;  // DMA pieces per row
  const unsigned loff = (unsigned)dma_lane_off<C, W>(lane) * 2u;
  // cursor over (stage l, image n, band b) and the band's first row R within this
  // workgroup's images ((n - n0) H + b BR, 32-bit): every address of a band is a per-stage
  // 64-bit base (computed once per stage) plus R times a power of two, so a band costs a
  // few scalar adds instead of 64-bit multiplies (the r05f instruction mix: ~180 scalar
  // instructions per band and wave before, a wave issues one instruction per ~4 cycles)
  int cl = 0, cn = n0, cb = 0, cR = 0;
  int xl = 0, xn = n0, xb = 0, xR = 0;  // next item
  auto adv = [&](int& l, int& n, int& b, int& R) {
    if (++b == nb) {
      b = 0;
      if (++n == n1) {
        n = n0;
        ++l;
        R = 0;
      } else {
        R = (n - n0) * H;
      }
    } else {
      R += BR;
    }
  };
  constexpr unsigned ROWBYTES = W * C * 2, MROWBYTES = W * C / 8;
  static_assert(ROWBYTES == 4096 && MROWBYTES == 256, "row byte shifts");
  const long img0 = (long)n0 * H;  // this workgroup's first image row
  const unsigned region = (unsigned)((n1 - n0) * H);  // its image rows
  // per stage: the output / mask buffer descriptors (base = this workgroup's first row) and
  // the next stage's DMA source base
  auto out_rs = [&](int st) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)(out_of(st) + img0 * W * C), 0, region * ROWBYTES, 0x00020000);
  };
  auto mask_rs = [&](int st) {
    uint8_t* m = mask_of(st);
    return __builtin_amdgcn_make_buffer_rsrc((void*)(m ? m + img0 * MROWBYTES : m), 0, m ? region * MROWBYTES : 0u,
                                             0x00020000);
  };
  auto src_base = [&](int st) { return (const unsigned char*)(src_of(st) + img0 * W * C); };
  adv(xl, xn, xb, xR);
  dma_rows<C, W>(x0, lds, cn, -1, min(BR, H) + 2, H, wave, NW, lane);
  int nst = 0;
  const int total = (RK2 ? 2 : 1) * L * per;
  ASR_BCLK(0, 0);
  int buf = 0, nbuf = 1, pbuf = NT - 1;  // this band's tile, the next band's, the previous band's
  auto yrs = out_rs(0);
  auto mrs = mask_rs(0);
  bool hasm = mask_of(0) != nullptr;
  const unsigned char* nsrc = src_base(0);  // the next item's stage's source rows
  int nsrc_st = 0;
  for (int it = 0; it < total; ++it) {
    if (wave == 0) ASR_BTR(0, 0, it, 0);
    barrier_vm_usual<2 * BR>(nst);  // band it landed; every wave is done with band it-1's tile
    if (wave == 0) ASR_BTR(0, 0, it, 1);
    nst = 0;
    // the next band into the ring: rows 0, 1 are this band's rows BR, BR+1 when it
    // continues the image (read in place), the rest by DMA
    if (it + 1 < total) {
      if (xl != nsrc_st) {  // (once per stage)
        nsrc = src_base(xl);
        nsrc_st = xl;
      }
      const int yy = xb * BR;
      const bool ncont = xl == cl && xn == cn && xb == cb + 1;
      const int r0 = ncont ? 1 : -1;  // image row offset of the first DMA'd tile row
      const int nrows = min(BR, H - yy) + (ncont ? 0 : 2);
      const unsigned nt0 = lds_u32(lds + nbuf * TILE) + (ncont ? 2u * BD::ROWB : 0u);
      // whole rows, one dma16x4 each (wave w: rows w, w + 4)
      for (int r = __builtin_amdgcn_readfirstlane(wave); r < nrows; r += NW) {
        const int gy = yy + r0 + r;
        const unsigned char* rowp = (unsigned)gy < (unsigned)H
                                        ? nsrc + (size_t)((unsigned)(xR + r0 + r) * ROWBYTES)
                                        : (const unsigned char*)g_zero_page;
        dma16x4_at(rowp + loff, nt0 + (unsigned)(r * BD::ROWB) + (unsigned)(NQ * 16));
      }
    }
    if (wave == 0) ASR_BTR(0, 0, it, 2);
    const unsigned tb = lds_u32(lds + buf * TILE);
    // input rows 0, 1: the previous band's tile rows BR, BR+1 when this band continues its image
    const unsigned th = cb > 0 ? lds_u32(lds + pbuf * TILE) + (unsigned)(BR * BD::ROWB) : tb;
    f32x4 acc[RB][2];
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int pt = 0; pt < 2; ++pt) acc[r][pt] = f32x4{bz[0], bz[1], bz[2], bz[3]};
    u32x4 xr[RB];
    const bool resg = RK2 && (cl & 1);  // second RK2 stage: residual x_l from global memory
    if (resg) {  // rows past the image end re-read its last row (never stored)
      const int y0 = cb * BR, rows = min(BR, H - y0);
      const unsigned char* rb = (const unsigned char*)(xin_of(cl >> 1) + ((long)cn * H + y0) * W * C) + ly;
#pragma unroll
      for (int r = 0; r < RB; ++r) xr[r] = *(const u32x4*)(rb + (long)min(r, rows - 1) * W * C * 2);
    }
    conv_band2<C, W, RB>(tb, th, lo, A, acc);
    if (wave == 0) ASR_BTR(0, 0, it, 3);
    if (!resg) {  // tile rows 1..RB (row 1 a halo row)
#pragma unroll
      for (int r = 0; r < RB; ++r) xr[r] = lds_rd128((r == 0 ? th : tb) + lxr + (unsigned)(r * BD::ROWB));
    }
    const int l = cl;
    if (blk_of(xl) != blk_of(cl) && it + 1 < total) {  // the next item starts block l+1: its W and bias (L2 hits)
      load_A1_untracked<C>(wpack + (long)blk_of(xl) * w_stride, ot, lane, A);
      load_bias4_untracked(bias ? bias + (long)blk_of(xl) * bias_stride + 16 * ot : nullptr, g, bz);
    }
    lgkm_wait<0>();
    const int rows = min(BR, H - cb * BR);
    // the band's y rows and mask rows as buffer stores: the stage's descriptor, the lane's
    // 32-bit offset and the row (R + r) as the scalar offset
    const float hst = (RK2 && !(l & 1)) ? 0.5f * h : h;
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      if (r >= rows) break;
      float z[8];
      regroup(acc[r][0], acc[r][1], z);
      u32x4 yw;
      unsigned bits = 0;
      static_for<0, 4>([&](auto dc) {
        constexpr int d = decltype(dc)::value;
        const int ra = max(__float_as_int(z[2 * d]), 0), rb = max(__float_as_int(z[2 * d + 1]), 0);
        yw[d] = pk_bf16(fmaf(hst, __int_as_float(ra), lo_f(xr[r][d])), fmaf(hst, __int_as_float(rb), hi_f(xr[r][d])));
        // relu-mask bits two at a time: [ra > 0] at bit 2d, [rb > 0] at bit 16 + 2d
        const unsigned pw = bits01_pair(ra, rb);
        bits = d == 0 ? pw : lshl_or<2 * d>(pw, bits);
      });
      bits = pair_bits_to_byte(bits);
      if (hasm) {
        __builtin_amdgcn_raw_buffer_store_b8((unsigned char)bits, mrs, (int)lm, (int)((unsigned)(cR + r) * MROWBYTES), 0);
        ++nst;
      }
      __builtin_amdgcn_raw_buffer_store_b128(yw, yrs, (int)ly, (int)((unsigned)(cR + r) * ROWBYTES), 0);
      ++nst;
    }
    if (wave == 0) ASR_BTR(0, 0, it, 4);
    if (xl != cl && it + 1 < total) {  // the next item starts a new stage: its store descriptors
      yrs = out_rs(xl);
      mrs = mask_rs(xl);
      hasm = mask_of(xl) != nullptr;
    }
    cl = xl, cn = xn, cb = xb, cR = xR;
    adv(xl, xn, xb, xR);
    pbuf = buf, buf = nbuf, nbuf = nbuf + 1 == NT ? 0 : nbuf + 1;
  }
  ASR_BCLK(0, 1);
}

// ===========================================================================
// fused backward
// ===========================================================================
template <int C, int W, int BR>
struct BwdLds {
  static constexpr int TW = W + 2;
  static constexpr int TILE = (BR + 2) * TW * (C / 8) * 16;
  static constexpr int RBM = W * C / 8;  // mask bytes per image row
  // mask bytes per buffer: the band's rows, or 2 copied rows + whole 1 KiB DMAs of the other BR
  static constexpr int MTB0 = ((BR + 2) * RBM + 1023) / 1024 * 1024;
  static constexpr int MTB1 = (2 * RBM + (BR * RBM + 1023) / 1024 * 1024 + 1023) / 1024 * 1024;
  static constexpr int MTB = MTB0 > MTB1 ? MTB0 : MTB1;
  static constexpr int DY = 0;                 // 2 x TILE (dy, halo rows)
  static constexpr int X = DY + 2 * TILE;      // 2 x TILE (x, halo rows)
  static constexpr int DZ = X + 2 * TILE;      // 1 x TILE (dz, halo rows)
  static constexpr int MSK = DZ + TILE;        // 2 x MTB
  static constexpr int TOTAL = MSK + 2 * MTB;
  // XT (RK2 first stage): per dgrad wave, a private copy of the extra dx
  // term for its MR rows x W pixels x its OTW o-tiles (NCH 16-B chunks/pixel)
  static constexpr int RS = 4 / Geo<C>::OSPLIT, MR = (BR + RS - 1) / RS;
  static constexpr int NCH = 2 * Geo<C>::OTW;
  static constexpr int ROWX = W * NCH * 16;    // bytes per private row
  static constexpr int EXT = TOTAL;            // 4 x MR x ROWX
  static constexpr int TOTAL_XT = EXT + 4 * MR * ROWX;
  static_assert(ROWX % 1024 == 0, "private extra rows are whole 1 KiB DMAs");
};

// DMA the extra dx term of one dgrad wave's rows (rg + k*RS) of the band at
// image row y0, its channels [16*OTW*oh, +16*OTW), into the wave's private
// rows: 16-B chunk j of pixel px sits in slot j ^ ((px / PXG) % NCH), PXG =
// the pixels one 64-bank span holds, so the epilogue's 8-B reads do not
// conflict.  Rows outside the band read the zero page.  Issues MR*ROWX/1024
// instructions.
template <int C, int W, int BR>
__device__ __forceinline__ void dma_extra(const bf16* __restrict__ extra, unsigned char* priv, int n, int y0, int rows,
                                          int H, int rg, int oh, int lane) {
  using L = BwdLds<C, W, BR>;
  constexpr int NCH = L::NCH, PXG = 64 / (NCH * 4);
#pragma unroll
  for (int k = 0; k < L::MR; ++k) {
    const int r = rg + k * L::RS;
#pragma unroll
    for (int q = 0; q < L::ROWX / 1024; ++q) {
      const int lb = q * 1024 + lane * 16;
      const int px = lb / (NCH * 16), slot = (lb / 16) % NCH;
      const int chunk = slot ^ ((px / PXG) % NCH);
      const void* src = (r < rows) ? (const void*)(extra + (((long)n * H + y0 + r) * W + px) * C +
                                                   16 * Geo<C>::OTW * oh + 8 * chunk)
                                   : (const void*)(g_zero_page + lane);
      dma16(src, priv + k * L::ROWX + q * 1024);
    }
  }
}

// The prefetch of the next band as one stream of 1 KiB DMA instructions
// [dy rows | x rows | mask chunks].  When the next band continues the same
// image, its two top tile rows are this band's two bottom rows: they are
// copied inside LDS (bwd_halo_copy) and the stream starts at tile row 2.
template <int C, int W, int BR, bool EULER>
struct BwdPrefetch {
  using L = BwdLds<C, W, BR>;
  static constexpr int IPR = W / Geo<C>::PPI, ROWB = (W + 2) * (C / 8) * 16;
  int n, gy0, nrows, ni, end;
  unsigned char *dyt, *xt, *mt;
  __device__ __forceinline__ void init(const ItemCursor& nx, bool active, bool reuse, unsigned char* lds, int buf, int H) {
    const int y0 = nx.b * BR, r0 = reuse ? 2 : 0;
    n = nx.n;
    gy0 = y0 - 1 + r0;
    nrows = min(BR, H - y0) + 2 - r0;
    ni = nrows * IPR;
    dyt = lds + L::DY + buf * L::TILE + r0 * ROWB;
    xt = lds + L::X + buf * L::TILE + r0 * ROWB;
    mt = lds + L::MSK + buf * L::MTB + r0 * L::RBM;
    end = active ? 2 * ni + (EULER ? (nrows * L::RBM + 1023) / 1024 : 0) : 0;
  }
  __device__ __forceinline__ void issue(int u, const bf16* dy, const bf16* x, const uint8_t* mask, int H, unsigned loff,
                                        int lane) const {
    if (u < ni)
      dma_row_instr<C, W>(dy, dyt, n, gy0, u, H, loff);
    else if (u < 2 * ni)
      dma_row_instr<C, W>(x, xt, n, gy0, u - ni, H, loff);
    else
      dma_mask_instr<C, W>(mask, mt, n, gy0, nrows, u - 2 * ni, H, lane);
  }
};

// tile rows BR, BR+1 of this band's dy/x tiles and mask rows -> rows 0, 1 of
// the next band's buffers (all threads; asm LDS accesses, see lds_rd128)
template <int C, int W, int BR, bool EULER>
__device__ __forceinline__ void bwd_halo_copy(unsigned char* lds, int buf, int tid, int nthreads) {
  using L = BwdLds<C, W, BR>;
  constexpr int ROWB = (W + 2) * (C / 8) * 16, NR = 2 * ROWB / 16, NM = EULER ? 2 * L::RBM / 16 : 0;
  constexpr int TOT = 2 * NR + NM, KB = (TOT + 511) / 512;
  const unsigned base = lds_u32(lds);
  u32x4 v[KB];
  unsigned dst[KB];
#pragma unroll
  for (int k = 0; k < KB; ++k) {
    const int c = tid + k * nthreads;
    const int cc = c < TOT ? c : 0;
    unsigned src;
    if (cc < NR) {
      src = L::DY + buf * L::TILE + BR * ROWB + cc * 16;
      dst[k] = L::DY + (buf ^ 1) * L::TILE + cc * 16;
    } else if (cc < 2 * NR) {
      src = L::X + buf * L::TILE + BR * ROWB + (cc - NR) * 16;
      dst[k] = L::X + (buf ^ 1) * L::TILE + (cc - NR) * 16;
    } else {
      src = L::MSK + buf * L::MTB + BR * L::RBM + (cc - 2 * NR) * 16;
      dst[k] = L::MSK + (buf ^ 1) * L::MTB + (cc - 2 * NR) * 16;
    }
    v[k] = lds_rd128(base + src);
  }
  lgkm_wait<0>();
#pragma unroll
  for (int k = 0; k < KB; ++k)
    if (tid + k * nthreads < TOT) lds_wr128(base + dst[k], v[k]);
}

template <int C, int W, int BR, bool EULER>
__device__ __forceinline__ void bwd_issue(const bf16* dy, const bf16* x, const uint8_t* mask, unsigned char* lds,
                                          int buf, int n, int y0, int H, int wave, int lane, int nwaves) {
  using L = BwdLds<C, W, BR>;
  const int nr = min(BR, H - y0) + 2;
  dma_rows<C, W>(dy, lds + L::DY + buf * L::TILE, n, y0 - 1, nr, H, wave, nwaves, lane);
  dma_rows<C, W>(x, lds + L::X + buf * L::TILE, n, y0 - 1, nr, H, wave, nwaves, lane);
  if constexpr (EULER) dma_mask_rows<C, W>(mask, lds + L::MSK + buf * L::MTB, n, y0 - 1, nr, H, wave, nwaves, lane);
}

// dzm = dy * mask for all staged rows, into the DZ tile: a bit operation on
// the bf16 values (the factor h of dz = h*dy*mask is applied in fp32 in the
// epilogues: dx, dW and db are linear in dz).  Interior columns only (the DZ
// tile's halo columns are zeroed once per launch), so chunk c of the band is
// (row, col, q) by shifts and its mask byte is byte c of the staged mask
// rows.  LDS accesses through asm (see lds_rd128): the dgrad waves run this
// with the next band's DMA in flight.
template <int C, int W, int BR, bool EULER>
__device__ __forceinline__ void bwd_convert(unsigned char* lds, int buf, int nr, int tid, int nthreads) {
  using L = BwdLds<C, W, BR>;
  constexpr int TW = W + 2, NQ = C / 8, KB = 4;
  static_assert((NQ & (NQ - 1)) == 0 && (W & (W - 1)) == 0, "power-of-two chunk decomposition");
  const unsigned dyt = lds_u32(lds + L::DY + buf * L::TILE);
  const unsigned mt = lds_u32(lds + L::MSK + buf * L::MTB);
  const unsigned dzt = lds_u32(lds + L::DZ);
  const int nch = nr * W * NQ;
  for (int c0 = tid; c0 < nch; c0 += KB * nthreads) {
    u32x4 v[KB];
    unsigned mb[KB];
    unsigned off[KB];
#pragma unroll
    for (int k = 0; k < KB; ++k) {  // all LDS reads first (latencies overlap)
      const int c = c0 + k * nthreads;
      const int cc = c < nch ? c : 0;
      const int q = cc & (NQ - 1), col = 1 + ((cc / NQ) & (W - 1)), r = cc / (NQ * W);
      off[k] = (unsigned)toff<C>(r, col, q, TW);
      v[k] = lds_rd128(dyt + off[k]);
      if constexpr (EULER) mb[k] = lds_rd_u8(mt + (unsigned)cc);
    }
    lgkm_wait<0>();
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      if (c0 + k * nthreads < nch) {
        u32x4 z = v[k];
        if constexpr (EULER) {
#pragma unroll
          for (int d = 0; d < 4; ++d) {  // element pair (2d, 2d+1) of this 16-byte chunk
            const unsigned lo = (unsigned)__builtin_amdgcn_sbfe((int)mb[k], 2 * d, 1);
            const unsigned hi = (unsigned)__builtin_amdgcn_sbfe((int)mb[k], 2 * d + 1, 1);
            z[d] &= __builtin_amdgcn_perm(hi, lo, 0x07060100u);  // bytes 0-1 of lo, 2-3 of hi
          }
        }
        lds_wr128(dzt + off[k], z);
      }
    }
  }
}

template <int C, int W, int BR, int MODE, bool XT>
__global__ __launch_bounds__(512) void k_bwd(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                             const uint8_t* __restrict__ mask, const bf16* __restrict__ wpack,
                                             float h, float two_gamma, int N, int H, bf16* __restrict__ dx,
                                             float* __restrict__ slabs, const bf16* __restrict__ extra,
                                             int skip_dy, int accum) {
  using G = Geo<C>;
  using L = BwdLds<C, W, BR>;
  constexpr int TW = W + 2, PT = W / 16, NQ = G::NQ, OTW = G::OTW, OT = G::OT, MTW = G::MTW;
  constexpr int KPR = W / 32;
  constexpr bool EULER = MODE == BWD_EULER;
  static_assert(W % 32 == 0, "wgrad k-steps are 32 pixels of one row");
  // XT: the RK2 variant (extra dx term and/or no +dy residual); compiled out
  // of the Euler block's kernel
  const bool has_extra = XT && extra != nullptr;
  const bool no_dy = XT && skip_dy != 0;
  // XT && accum: add to the slab this WG's slot already holds (the RK2 first
  // stage onto the second stage's slabs: same grid, so one slab set per block)
  const bool acc_slab = XT && accum != 0;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, lx = lane & 15;

  for (int b = 0; b < 2; ++b) {
    zero_halo_cols<C, W>(lds + L::DY + b * L::TILE, BR + 2, tid, 512);
    zero_halo_cols<C, W>(lds + L::X + b * L::TILE, BR + 2, tid, 512);
  }
  zero_halo_cols<C, W>(lds + L::DZ, BR + 2, tid, 512);
  const int nb = (H + BR - 1) / BR;
  int i0, i1;
  item_range(N * nb, &i0, &i1);
  if (i0 < i1) {
    const ItemCursor c0(i0, nb);
    bwd_issue<C, W, BR, EULER>(dy, x, mask, lds, 0, c0.n, c0.b * BR, H, wave, lane, 8);
  }

  float* slab = slabs + (long)blockIdx.x * (9 * C * C + C);
  const float hs = EULER ? h : 1.f;  // dz = hs * dzm (dzm = dy*mask in LDS)
  const float hs2g = hs * two_gamma;
  if (wave < 4) {
    // ---------------- dgrad waves ----------------
    constexpr int RS = 4 / G::OSPLIT;
    const int oh = wave % G::OSPLIT, rg = wave / G::OSPLIT;
    const int wv4 = __builtin_amdgcn_readfirstlane(wave);
    const unsigned loff = (unsigned)dma_lane_off<C, W>(lane) * 2u;
    bf16x8 A[OTW][G::KS];
    load_A<C>(wpack, oh, lane, A);
    Frag<C, W> boff;
    boff.init(g, lx);
    float dbacc[OTW][4];  // db partial for channels 16*(oh*OTW+t) + 4g + e over this lane's pixels
#pragma unroll
    for (int t = 0; t < OTW; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) dbacc[t][e] = 0.f;
    int nst = 0;
    // the extra dx term (RK2: the outer dy of the first stage): each dgrad
    // wave DMAs the rows it needs into its private LDS rows after its last
    // epilogue of the previous band (prologue: before the loop), so it is
    // older than the next band's prefetch and vm_wait(nd) covers it
    using LX = BwdLds<C, W, BR>;
    constexpr int MR = LX::MR, NEX = MR * LX::ROWX / 1024;
    unsigned char* priv = lds + LX::EXT + wave * MR * LX::ROWX;
    if (has_extra && i0 < i1) {
      const ItemCursor c0(i0, nb);
      dma_extra<C, W, BR>(extra, priv, c0.n, c0.b * BR, min(BR, H - c0.b * BR), H, rg, oh, lane);
      nst = NEX;
    }
    ItemCursor cur(i0, nb), nxt(i0, nb);
    nxt.next(nb);
    for (int it = i0; it < i1; ++it, cur.next(nb), nxt.next(nb)) {
      const int buf = (it - i0) & 1;
      const int n = cur.n, y0 = cur.b * BR;
      const int rows = min(BR, H - y0);
      ASR_STAMP(it - i0, 0);
      barrier_vm(nst);  // item's DMA landed; previous item fully consumed
      ASR_STAMP(it - i0, 1);
      nst = 0;
      // prefetch of band it+1: dy rows, x rows, mask chunks as one stream of
      // instructions dealt round-robin to all 8 waves; a dgrad wave issues
      // its share one per k-step of its first dgrad row (so the issue cost
      // overlaps MFMAs), the rest flushed before that row's epilogue
      int nd = 0;  // prefetch instructions this wave issued
      const bool reuse = it + 1 < i1 && nxt.n == cur.n;
      BwdPrefetch<C, W, BR, EULER> pf;
      pf.init(nxt, it + 1 < i1, reuse, lds, buf ^ 1, H);
      const int dsplit = (pf.end * kBwdDgradDmaPct) / 100;  // dgrad waves: [0, dsplit)
      int du = wv4;                                               // wave-uniform stream cursor
      const int dend = dsplit;
      auto dma_one = [&]() {
        if (du < dend) {
          pf.issue(du, dy, x, mask, H, loff, lane);
          du += 4;
          nst = 0;  // the next barrier waits for this prefetch; stores issued after it need not finish
          ++nd;
        }
      };
      bool ex_wait = has_extra;
      if (reuse) bwd_halo_copy<C, W, BR, EULER>(lds, buf, tid, 512);
      bwd_convert<C, W, BR, EULER>(lds, buf, rows + 2, tid, 512);
      ASR_STAMP(it - i0, 2);
      barrier_lds();  // dz ready
      ASR_STAMP(it - i0, 3);
      const unsigned char* dzt = lds + L::DZ;
      const unsigned char* dyt = lds + L::DY + buf * L::TILE;
#pragma unroll
      for (int k = 0; k < MR; ++k) {
        const int r = rg + k * RS;
        if (r >= rows) break;
        f32x4 acc[OTW][PT];
#pragma unroll
        for (int t = 0; t < OTW; ++t)
#pragma unroll
          for (int pt = 0; pt < PT; ++pt) acc[t][pt] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (k == 0) {
          conv_row<C, W>(dzt, r, A, boff, acc, dma_one);
          while (du < dend) dma_one();
          ASR_STAMP(it - i0, 4);
        } else {
          conv_row<C, W>(dzt, r, A, boff, acc);
        }
        const int gy = y0 + r;
        if (dx) nst += PT * OTW;
        u32x2 dzv[PT][OTW], dyv[PT][OTW];
#pragma unroll
        for (int pt = 0; pt < PT; ++pt)
#pragma unroll
          for (int t = 0; t < OTW; ++t) {
            const int px = 16 * pt + lx, o0 = 16 * (oh * OTW + t) + 4 * g;
            const int co = toff<C>(r + 1, px + 1, o0 >> 3, TW) + (o0 & 4) * 2;
            dzv[pt][t] = lds_rd64(lds_u32(dzt + co));
            if (EULER && !no_dy) dyv[pt][t] = lds_rd64(lds_u32(dyt + co));
          }
        lgkm_wait<0>();
        if (ex_wait) {
          vm_wait(nd);  // this wave's private extra rows (older than the next band's prefetch)
          ex_wait = false;
        }
#pragma unroll
        for (int pt = 0; pt < PT; ++pt) {
          const int px = 16 * pt + lx;
#pragma unroll
          for (int t = 0; t < OTW; ++t) {
            const int o0 = 16 * (oh * OTW + t) + 4 * g;
            const bf16x4 dzr = *(const bf16x4*)&dzv[pt][t];
            float dzf[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              dzf[e] = (float)dzr[e];
              dbacc[t][e] += dzf[e];
            }
            // residual terms: dy (unless skip_dy) + extra
            float res[4] = {0.f, 0.f, 0.f, 0.f};
            if (EULER && !no_dy) {
              const bf16x4 dyr = *(const bf16x4*)&dyv[pt][t];
#pragma unroll
              for (int e = 0; e < 4; ++e) res[e] = (float)dyr[e];
            }
            if (has_extra) {
              constexpr int PXG = 64 / (LX::NCH * 4);
              const int px = 16 * pt + lx;
              const unsigned a = lds_u32(priv + k * LX::ROWX + px * LX::NCH * 16 +
                                         (((2 * t + (g >> 1)) ^ ((px / PXG) % LX::NCH)) * 16) + (g & 1) * 8);
              u32x2 ev = lds_rd64(a);
              lgkm_wait<0>();
              const bf16x4 exr = *(const bf16x4*)&ev;
#pragma unroll
              for (int e = 0; e < 4; ++e) res[e] += (float)exr[e];
            }
            bf16x4 o4;
            if constexpr (EULER) {
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const float v = fmaf(-hs, acc[t][pt][e], res[e]);
                o4[e] = (bf16)(hs2g != 0.f ? fmaf(hs2g, dzf[e], v) : v);
              }
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e) o4[e] = (bf16)(fmaf(two_gamma, dzf[e], -acc[t][pt][e]) + res[e]);
            }
            if (dx) *(bf16x4*)(dx + (((long)n * H + gy) * W + px) * C + o0) = o4;
          }
        }
        ASR_STAMP(it - i0, 5 + k);
      }
      while (du < dend) dma_one();  // a wave without rows in this band
      if (has_extra && it + 1 < i1) {  // next band's extra rows into the (now read) private rows
        dma_extra<C, W, BR>(extra, priv, nxt.n, nxt.b * BR, min(BR, H - nxt.b * BR), H, rg, oh, lane);
        nst += NEX;
      }
    }
    // reduce db over the 16 pixel lanes, then over the row-group waves (LDS)
#pragma unroll
    for (int t = 0; t < OTW; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = dbacc[t][e];
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 4);
        v += __shfl_xor(v, 8);
        dbacc[t][e] = v;
      }
    barrier_vm(0);  // matches the wgrad waves' end-of-loop barrier
    float* dbl = (float*)lds + 12288;  // [RS][C], past the K-split scratch
    if (lx == 0) {
#pragma unroll
      for (int t = 0; t < OTW; ++t)
#pragma unroll
        for (int e = 0; e < 4; ++e) dbl[rg * C + 16 * (oh * OTW + t) + 4 * g + e] = hs * dbacc[t][e];
    }
    if constexpr (G::KSPLIT > 1) {
      __syncthreads();
      __syncthreads();
    }
  } else {
    // ---------------- wgrad waves ----------------
    const int w4 = wave - 4;
    const int tg = w4 % G::TG, kg = w4 / G::TG;
    const int tq = lx >> 2, tp = lx & 3;
    f32x4 acc[MTW][OT];
#pragma unroll
    for (int mi = 0; mi < MTW; ++mi)
#pragma unroll
      for (int ot = 0; ot < OT; ++ot) acc[mi][ot] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int wv8 = __builtin_amdgcn_readfirstlane(wave);
    const unsigned loff = (unsigned)dma_lane_off<C, W>(lane) * 2u;
    ItemCursor cur(i0, nb), nxt(i0, nb);
    nxt.next(nb);
    for (int it = i0; it < i1; ++it, cur.next(nb), nxt.next(nb)) {
      const int buf = (it - i0) & 1;
      const int y0 = cur.b * BR;
      const int rows = min(BR, H - y0);
      ASR_STAMP(it - i0, 0);
      barrier_vm(0);  // this wave's share of the band's prefetch landed (no stores in flight)
      ASR_STAMP(it - i0, 1);
      // this wave's share of band it+1's prefetch (see the dgrad waves),
      // issued after the dz barrier, while the dgrad wave on this SIMD runs
      // its MFMAs
      const bool reuse = it + 1 < i1 && nxt.n == cur.n;
      BwdPrefetch<C, W, BR, EULER> pf;
      pf.init(nxt, it + 1 < i1, reuse, lds, buf ^ 1, H);
      int du = (pf.end * kBwdDgradDmaPct) / 100 + wv8 - 4;  // wgrad waves: [dsplit, end)
      const int dend = pf.end;
      auto dma_one = [&]() {
        if (du < dend) {
          pf.issue(du, dy, x, mask, H, loff, lane);
          du += 4;
        }
      };
      if (reuse) bwd_halo_copy<C, W, BR, EULER>(lds, buf, tid, 512);
      bwd_convert<C, W, BR, EULER>(lds, buf, rows + 2, tid, 512);
      ASR_STAMP(it - i0, 2);
      barrier_lds();
      ASR_STAMP(it - i0, 3);
      while (du < dend) dma_one();
      ASR_STAMP(it - i0, 4);
      const unsigned char* dzt = lds + L::DZ;
      const unsigned char* xt = lds + L::X + buf * L::TILE;
      for (int kk = kg; kk < rows * KPR; kk += G::KSPLIT) {
        const int r = kk / KPR, kb = kk % KPR;
        const int pb = 32 * kb + 8 * g + tq;
        auto loadA = [&](int mi) {
          const int mt = tg * MTW + mi;
          const int tap = (16 * mt) / C, itile = ((16 * mt) % C) / 16;
          const int ky = tap / 3, kx = tap % 3;
          const int q = 2 * itile + (tp >> 1);
          return tr_pair(xt + toff<C>(r + ky, pb + kx, q, TW) + 8 * (tp & 1),
                         xt + toff<C>(r + ky, pb + 4 + kx, q, TW) + 8 * (tp & 1));
        };
        bf16x8 Bf[OT];
#pragma unroll
        for (int ot = 0; ot < OT; ++ot) {
          const int q = 2 * ot + (tp >> 1);
          Bf[ot] = tr_pair(dzt + toff<C>(r + 1, pb + 1, q, TW) + 8 * (tp & 1),
                           dzt + toff<C>(r + 1, pb + 5, q, TW) + 8 * (tp & 1));
        }
        bf16x8 Ac = loadA(0), An;
#pragma unroll
        for (int mi = 0; mi < MTW; ++mi) {
          if (mi + 1 < MTW) An = loadA(mi + 1);
#pragma unroll
          for (int ot = 0; ot < OT; ++ot)
            acc[mi][ot] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ac, Bf[ot], acc[mi][ot], 0, 0, 0);
          if (mi + 1 < MTW) Ac = An;
        }
      }
      ASR_STAMP(it - i0, 5);
    }
    barrier_vm(0);  // all items consumed: LDS reusable
    float* red = (float*)lds;
    if constexpr (G::KSPLIT > 1) {
      if (kg > 0) {
#pragma unroll
        for (int mi = 0; mi < MTW; ++mi)
#pragma unroll
          for (int ot = 0; ot < OT; ++ot)
#pragma unroll
            for (int e = 0; e < 4; ++e)
              red[((((kg - 1) * G::TG + tg) * MTW + mi) * OT + ot) * 256 + e * 64 + lane] = acc[mi][ot][e];
      }
      __syncthreads();
      if (kg == 0) {
        for (int k2 = 1; k2 < G::KSPLIT; ++k2)
#pragma unroll
          for (int mi = 0; mi < MTW; ++mi)
#pragma unroll
            for (int ot = 0; ot < OT; ++ot)
#pragma unroll
              for (int e = 0; e < 4; ++e)
                acc[mi][ot][e] += red[((((k2 - 1) * G::TG + tg) * MTW + mi) * OT + ot) * 256 + e * 64 + lane];
      }
      __syncthreads();
    }
    if (kg == 0) {
      // acc_slab: the old values of MC m-tiles loaded before their first
      // store (one latency per chunk, not one per element: the compiler keeps
      // load/store pairs to the slab in order)
      constexpr int MC = MTW % 3 == 0 ? 3 : 1;
#pragma unroll
      for (int m0 = 0; m0 < MTW; m0 += MC) {
        float prev[MC][OT][4];
#pragma unroll
        for (int mi = 0; mi < MC; ++mi)
#pragma unroll
          for (int ot = 0; ot < OT; ++ot)
#pragma unroll
            for (int e = 0; e < 4; ++e)
              prev[mi][ot][e] =
                  acc_slab ? slab[(long)(16 * (tg * MTW + m0 + mi) + 4 * g + e) * C + 16 * ot + lx] : 0.f;
#pragma unroll
        for (int mi = 0; mi < MC; ++mi)
#pragma unroll
          for (int ot = 0; ot < OT; ++ot)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int m = 16 * (tg * MTW + m0 + mi) + 4 * g + e;
              slab[(long)m * C + 16 * ot + lx] = fmaf(hs, acc[m0 + mi][ot][e], prev[mi][ot][e]);
            }
      }
    }
  }
  __syncthreads();
  if (tid < C) {
    const float* dbl = (const float*)lds + 12288;
    float s = 0.f;
    for (int q = 0; q < 4 / G::OSPLIT; ++q) s += dbl[q * C + tid];
    slab[9 * C * C + tid] = acc_slab ? slab[9 * C * C + tid] + s : s;
  }
}

// ===========================================================================
// Backward v2 (C=64, W=32, BR=4; the Euler block and the plain conv, no
// RK2 extra term).  The dz = dy*mask conversion of band it+1 runs on the
// dgrad waves at the end of band it, while the wgrad waves still run band
// it's MFMAs (v1 converts on all 8 waves between two barriers, with the MFMA
// pipe idle).  dy, x and dz tiles are double-buffered (6 tiles, 153 KiB);
// the relu mask goes to registers, not LDS.  Each dgrad wave owns whole
// tile rows of the next band: it DMAs their dy, loads their mask dwords and
// converts them, so its own vmcnt covers everything it converts and no
// cross-wave wait is needed before the band barrier.  The wgrad waves DMA
// the next band's x rows and, after their MFMAs, copy the halo rows of a
// band that continues the previous band's image (dz rows 0,1 already
// masked, x rows 0,1, dy row 1 = the residual's first interior row).
// ===========================================================================
template <int C, int W, int BR>
struct Bwd2Lds {
  static constexpr int ROWB = (W + 2) * (C / 8) * 16;
  static constexpr int TILE = (BR + 2) * ROWB;
  static constexpr int DY = 0, X = 2 * TILE, DZ = 4 * TILE;
  // 256 x 16 B: the 16-bit-lane AND masks of one 16-B chunk per mask byte
  static constexpr int MTAB = 6 * TILE, TOTAL = MTAB + 4096;
};

// tile rows of band `nx` owned by dgrad wave wv (0..3): reuse -> row 2+wv;
// else rows wv and wv+4 (wv < 2)
struct Bwd2Own {
  int ra, rb;  // rb < 0: one row
  __device__ __forceinline__ Bwd2Own(bool reuse, int wv) {
    ra = reuse ? 2 + wv : wv;
    rb = (!reuse && wv < 2) ? wv + 4 : -1;
  }
  __device__ __forceinline__ int count() const { return rb < 0 ? 1 : 2; }
  __device__ __forceinline__ int row(int k) const { return k == 0 ? ra : rb; }
};

// mask dword of lane (pixel lane&31, channel half lane>>5) of tile row r of
// band (n, y0): bytes 8*px + 4*h .. +3 of the image row (zeros outside)
template <int C, int W>
__device__ __forceinline__ unsigned bwd2_mask_word(const uint8_t* __restrict__ mask, int n, int y0, int r, int H,
                                                   int lane) {
  const int gy = y0 - 1 + r;
  if ((unsigned)gy >= (unsigned)H) return 0u;
  return *(const unsigned*)(mask + ((long)n * H + gy) * (W * C / 8) + (2 * (lane & 31) + (lane >> 5)) * 4);
}


// ===========================================================================
// Backward v3 (C=64, W=32, BR=4): the round-1 v2 backward's band protocol (double-buffered
// dy / x / dz tiles, the next band's dz converted by the dgrad waves from
// their own dy rows, x DMA + halo copy by the wgrad waves, the previous
// block's slab pass folded in) at three waves per SIMD (12 waves, <= 168
// VGPRs):
//   waves 0-3  dgrad, one 16-channel o-tile each over the whole band (the
//              forward's band conv on the dz tile: A 72 VGPRs), epilogue on
//              the regrouped accumulators (16-B dy / dz / x chunk reads, one
//              16-B dx store per row, db over 8 channels per lane);
//   waves 4-11 wgrad, m-tile group tg = (w-4)/2 (9 m-tiles) x o-tiles
//              2*((w-4)&1) + 0..1: 72 accumulator VGPRs, 18 MFMAs per k-step.
// dW sums the pixels of a row in a bank-conflict-free permutation, dx the taps
// in the band conv's order, db on MFMA.
// ===========================================================================
template <int C, int W, int BR, int MODE, bool RO, bool XT = false>
__global__ __launch_bounds__(768, 1) void k_bwd3(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                 const uint8_t* __restrict__ mask, const bf16* __restrict__ wpack,
                                                 float h, float two_gamma, int N, int H, bf16* __restrict__ dx,
                                                 float* __restrict__ slabs, const float* __restrict__ pslabs, int pP,
                                                 float* __restrict__ pgrp, int skip_dy,
                                                 const bf16* __restrict__ extra = nullptr) {
  using G = Geo<C>;
  using L = Bwd2Lds<C, W, BR>;
  using BD = Band<C, W, BR>;
  constexpr int TW = W + 2, OT = G::OT, MTW = G::MTW, IPR = W / G::PPI, NQ = G::NQ;
  constexpr bool EULER = MODE == BWD_EULER;
  static_assert(C == 64 && W == 32 && BR == 4 && MTW == 9 && OT == 4, "v3 backward geometry");
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, lx = lane & 15;

  for (int b = 0; b < 2; ++b) {
    zero_halo_cols<C, W>(lds + L::DY + b * L::TILE, BR + 2, tid, 768);
    zero_halo_cols<C, W>(lds + L::X + b * L::TILE, BR + 2, tid, 768);
    zero_halo_cols<C, W>(lds + L::DZ + b * L::TILE, BR + 2, tid, 768);
  }
  if (EULER) {  // dword d of byte m's entry: 0xffff per set bit of (m >> 2d) & 3
    unsigned* tab = (unsigned*)(lds + L::MTAB);
    for (int i = tid; i < 1024; i += 768) {
      const unsigned m = (unsigned)i >> 2, d = (unsigned)i & 3;
      tab[i] = (((m >> (2 * d)) & 1u) ? 0xffffu : 0u) | (((m >> (2 * d + 1)) & 1u) ? 0xffff0000u : 0u);
    }
  }
  const int nb = (H + BR - 1) / BR;
  int i0, i1;
  item_range(N * nb, &i0, &i1);
  const unsigned loff = (unsigned)dma_lane_off<C, W>(lane) * 2u;
  float* slab = slabs + (long)blockIdx.x * (9 * C * C + C);
  const float hs = EULER ? h : 1.f;  // dz = hs * dzm (dzm = dy*mask in LDS)
  const float hs2g = hs * two_gamma;
  __syncthreads();  // halo columns zeroed before any convert / copy writes near them
  ASR_BCLK(1, 0);

  // pass 1 of the previous block's slab reduction (as in the round-1 v2 backward), on the wgrad
  // waves only: thread ft = tid - 256 owns one 16-B chunk of one group row
  constexpr int ES = 9 * C * C + C, ECH = ES / 4;
  const int ft = tid - 256;
  const long fT = (long)((pP + 31) / 32) * ECH;
  const long fc0 = (long)blockIdx.x * fT / gridDim.x, fc1 = (long)(blockIdx.x + 1) * fT / gridDim.x;
  const bool fold = pP > 0 && ft >= 0 && fc0 + ft < fc1;
  const int fg = fold ? (int)((fc0 + ft) / ECH) : 0;
  const int fpe = min(pP, 32 * fg + 32);
  int fp = 32 * fg;
  unsigned foff = fold ? (unsigned)fp * ES + (unsigned)((fc0 + ft) % ECH) * 4 : 0u;
  f32x4 facc = {0.f, 0.f, 0.f, 0.f}, fv[2];

  if (wave < 4) {
    // ---------------- dgrad waves ----------------
    const int ot = wave;
    bf16x8 A[G::KS];
    load_A1<C>(wpack, ot, lane, A);
    unsigned lo[3 * BD::NCB];
    band_lane_offsets<C, W, BR>(g, lx, lo);
    const int px = lx + 16 * (g & 1), cg = 2 * ot + (g >> 1);  // regrouped: pixel, 16-B channel chunk
    const unsigned lch = (unsigned)toff<C>(1, px + 1, cg, TW);  // output row 0's chunk in a tile
    const unsigned ldx = (unsigned)(px * C + 8 * cg) * 2u;
    int nst = 0;
    ItemCursor cur(i0, nb);
    for (int it = i0; it < i1; ++it, cur.next(nb)) {
      const int buf = (it - i0) & 1;
      const int n = cur.n, y0 = cur.b * BR;
      const int rows = min(BR, H - y0);
      if (wave == 0) ASR_BTR(1, 0, it - i0, 0);
      barrier_vm_usual<BR>(nst);  // band it staged everywhere; band it-1 fully consumed
      if (wave == 0) ASR_BTR(1, 0, it - i0, 1);
      // XT: the extra dx term of the band's rows (in flight during the conv)
      u32x4 exv[XT ? BR : 1];
      if constexpr (XT) {
        const bf16* eb = extra + ((long)n * H + y0) * W * C;
#pragma unroll
        for (int r = 0; r < BR; ++r) {
          const int rr = min(r, rows - 1);
          exv[r] = *(const u32x4*)((const unsigned char*)(eb + (long)rr * W * C) + ldx);
        }
      }
      const unsigned dzt = lds_u32(lds + L::DZ + buf * L::TILE), dyt = lds_u32(lds + L::DY + buf * L::TILE);
      const unsigned xt = lds_u32(lds + L::X + buf * L::TILE);
      f32x4 acc[BR][2];
#pragma unroll
      for (int r = 0; r < BR; ++r) acc[r][0] = acc[r][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (wave == 0) ASR_BTR(1, 0, it - i0, 2);
      conv_band<C, W, BR>(dzt, lo, A, acc);
      if (wave == 0) ASR_BTR(1, 0, it - i0, 3);
      // epilogue, LDS reads one row ahead: dy (the residual), dz only for the
      // 2*gamma*dz term (gamma != 0), x for RO; the flags are compile-time in
      // each instantiation (a runtime flag costs selects on every element)
      bf16* drow = dx ? dx + ((long)n * H + y0) * W * C : nullptr;
      int nld = 0;
      auto epilogue = [&](auto g2c, auto skc) {
        constexpr bool G2 = decltype(g2c)::value, SKIP = decltype(skc)::value;
        constexpr bool RDY = EULER && !SKIP;
        constexpr int NR = (RDY ? 1 : 0) + (G2 ? 1 : 0) + (RO ? 1 : 0);  // LDS reads per row
        u32x4 dyw[2], dzw[2], xw[2];
        auto issue = [&](int r, int sl) {
          const unsigned co = lch + (unsigned)(r * L::ROWB);
          if constexpr (RDY) dyw[sl] = lds_rd128(dyt + co);
          if constexpr (G2) dzw[sl] = lds_rd128(dzt + co);
          if constexpr (RO) xw[sl] = lds_rd128(xt + co);
        };
        // reads of all BR tile rows on a compile-time schedule (rows past the image
        // read tile rows that exist and are not used), each retired before the row
        // guard: no branch between a read and its wait (see k_bwd3_stack)
        if constexpr (NR > 0) issue(0, 0);
        static_for<0, BR>([&](auto rc) {
          constexpr int r = decltype(rc)::value, sl = r & 1;
          if constexpr (NR > 0) {
            if constexpr (r + 1 < BR) {
              issue(r + 1, sl ^ 1);
              lgkm_wait<NR>();  // row r's reads (row r+1's still in flight)
            } else {
              lgkm_wait<0>();
            }
          }
          if (r < rows) {
            float z[8];
            regroup(acc[r][0], acc[r][1], z);
            u32x4 ow;
#pragma unroll
            for (int d = 0; d < 4; ++d) {
              float v0, v1;
              if constexpr (EULER) {
                float r0 = 0.f, r1 = 0.f;
                if constexpr (RDY) r0 = lo_f(dyw[sl][d]), r1 = hi_f(dyw[sl][d]);
                if constexpr (XT) {
                  r0 += lo_f(exv[r][d]);
                  r1 += hi_f(exv[r][d]);
                }
                v0 = fmaf(-hs, z[2 * d], r0);
                v1 = fmaf(-hs, z[2 * d + 1], r1);
                if constexpr (G2) {
                  v0 = fmaf(hs2g, lo_f(dzw[sl][d]), v0);
                  v1 = fmaf(hs2g, hi_f(dzw[sl][d]), v1);
                }
              } else {
                v0 = -z[2 * d];
                v1 = -z[2 * d + 1];
                if constexpr (G2) {
                  v0 = fmaf(two_gamma, lo_f(dzw[sl][d]), v0);
                  v1 = fmaf(two_gamma, hi_f(dzw[sl][d]), v1);
                }
              }
              ow[d] = pk_bf16(v0, v1);
              if constexpr (RO) {  // bf16 x > 0: positive as a signed 16-bit integer
                const unsigned xd = xw[sl][d];
                ow[d] &= ((int)(short)(xd & 0xffffu) > 0 ? 0xffffu : 0u) | ((int)xd > 0xffff ? 0xffff0000u : 0u);
              }
            }
            if (drow) {
              *(u32x4*)((unsigned char*)(drow + (long)r * W * C) + ldx) = ow;
              ++nld;
            }
          }
        });
      };
      using T_ = std::true_type;
      using F_ = std::false_type;
      const bool g2 = hs2g != 0.f;
      if (EULER && skip_dy) {
        if (g2) epilogue(T_{}, T_{});
        else epilogue(F_{}, T_{});
      } else {
        if (g2) epilogue(T_{}, F_{});
        else epilogue(F_{}, F_{});
      }
      if (wave == 0) ASR_BTR(1, 0, it - i0, 4);
      if (wave == 0) ASR_BTR(1, 0, it - i0, 5);
      nst = nld;
    }
    barrier_vm(0);  // matches the wgrad waves' end-of-loop barrier
  } else {
    // ---------------- wgrad waves ----------------
    const int w8 = __builtin_amdgcn_readfirstlane(wave) - 4;
    const int tg = w8 >> 1, oq = 2 * (w8 & 1);  // m-tiles tg*9 .. +8, o-tiles oq, oq+1
    const int tq = lx >> 2, tp = lx & 3;
    f32x4 acc[MTW][2];
#pragma unroll
    for (int mi = 0; mi < MTW; ++mi) acc[mi][0] = acc[mi][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    // per-lane byte offsets (tile row 0) of the transposed fragment reads:
    // A = x at tap (ky, kx) of m-tile tg*9 + mi, B = dz of o-tile oq + oi (output row 0 = tile row 1)
    // LDS byte addresses in the current band's buffer (row r's r * ROWB is an immediate).
    // K = the row's 32 pixels, lane group g reading pixels 4g + tq and 4g + 16 + tq
    // (any pixel permutation shared by A and B gives the same GEMM): each 32-lane
    // half then reads 8 consecutive tile columns, whose swizzled 8-B pieces cover
    // the 64 banks once (pixels 8g + tq, 8g + 4 + tq, as the round-1 v2 backward read them, put
    // columns c and c + 8 on the same banks: every read 2-way)
    unsigned offA[MTW], offB[2];  // pixel tile 1 sits 16 px = 2 KiB on (swizzle period 8 px)
    {
      const unsigned xb0 = lds_u32(lds + L::X), zb0 = lds_u32(lds + L::DZ);
      const int pb = 4 * g + tq;
#pragma unroll
      for (int mi = 0; mi < MTW; ++mi) {
        const int mt = tg * MTW + mi;
        const int tap = (16 * mt) / C, itile = ((16 * mt) % C) / 16;
        const int ky = tap / 3, kx = tap % 3, q = 2 * itile + (tp >> 1);
        offA[mi] = xb0 + (unsigned)(toff<C>(ky, pb + kx, q, TW) + 8 * (tp & 1));
      }
#pragma unroll
      for (int oi = 0; oi < 2; ++oi) {
        const int q = 2 * (oq + oi) + (tp >> 1);
        offB[oi] = zb0 + (unsigned)(toff<C>(1, pb + 1, q, TW) + 8 * (tp & 1));
      }
      // opaque to the compiler: kept in VGPRs, not recomputed per band
#pragma unroll
      for (int mi = 0; mi < MTW; ++mi) asm volatile("" : "+v"(offA[mi]));
      asm volatile("" : "+v"(offB[0]), "+v"(offB[1]));
    }
    // the next band's dz: wgrad wave w8 owns tile row 2 + w8 (w8 < 4) of a band that
    // continues the image, row w8 (w8 < 6) of one that starts an image; it DMAs
    // that row's dy, loads its mask dwords and converts it (its own vmcnt covers both)
    auto own_row = [&](bool reuse) { return reuse ? (w8 < 4 ? 2 + w8 : -1) : (w8 < 6 ? w8 : -1); };
    auto stage_own = [&](const ItemCursor& c, int row, int nbuf, unsigned& mwv) {
      if (row < 0) return;
      if constexpr (EULER) mwv = bwd2_mask_word<C, W>(mask, c.n, c.b * BR, row, H, lane);
      for (int j = 0; j < IPR; ++j)
        dma_row_instr<C, W>(dy, lds + L::DY + nbuf * L::TILE + row * L::ROWB, c.n, c.b * BR - 1 + row, j, H, loff);
    };
    // dz = dy & mask of the own row (lane = pixel lane&31, chunks 4*(lane>>5) + j),
    // two chunks at a time, compiler-visible LDS accesses (this role's live state
    // leaves little room: a spilled inline-asm read result would be garbage)
    auto convert_own = [&](int row, int nbuf, unsigned mwv) {
      if (row < 0) return;
      const unsigned base = lds_u32(lds);
      const int cpx = lane & 31, hh = lane >> 5;
#pragma unroll
      for (int jj = 0; jj < 4; jj += 2) {
        u32x4 v[2], mt[2];
        unsigned off[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          off[j] = (unsigned)toff<C>(row, cpx + 1, 4 * hh + jj + j, TW) + (unsigned)(nbuf * L::TILE);
          v[j] = lds_ld128(base + L::DY + off[j]);
          if (EULER) mt[j] = lds_ld128(base + L::MTAB + __builtin_amdgcn_ubfe(mwv, 8 * (jj + j), 8) * 16);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          u32x4 z = v[j];
          if constexpr (EULER) {
            z &= mt[j];
          } else if constexpr (EULER) {
#pragma unroll
            for (int d = 0; d < 4; ++d) {
              const unsigned lo = (unsigned)__builtin_amdgcn_sbfe((int)mwv, 8 * (jj + j) + 2 * d, 1);
              const unsigned hi = (unsigned)__builtin_amdgcn_sbfe((int)mwv, 8 * (jj + j) + 2 * d + 1, 1);
              z[d] &= __builtin_amdgcn_perm(hi, lo, 0x07060100u);
            }
          }
          lds_st128(base + L::DZ + off[j], z);
        }
      }
    };
    // db on MFMA (tile group 3): ones(16 x 32) x dz^T, every row of the result = db
    bf16x8 ones;
#pragma unroll
    for (int i = 0; i < 8; ++i) ones[i] = (bf16)1.0f;
    f32x4 accb[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    const bool dbw = tg == 3;
    if (i0 < i1) {  // prologue: dy rows (own) and x rows of band i0, its dz converted
      const ItemCursor c0(i0, nb);
      unsigned mw0 = 0u;
      const int row0 = own_row(false);
      stage_own(c0, row0, 0, mw0);
      for (int j = w8; j < (BR + 2) * IPR; j += 8) dma_row_instr<C, W>(x, lds + L::X, c0.n, c0.b * BR - 1, j, H, loff);
      // (the band loop's x DMA runs on waves w8 >= 4 only: waves 0-3 DMA the own dy rows)
      vm_wait(0);
      convert_own(row0, 0, mw0);
    }
    ItemCursor cur(i0, nb), nxt(i0, nb);
    nxt.next(nb);
    for (int it = i0; it < i1; ++it, cur.next(nb), nxt.next(nb)) {
      const int buf = (it - i0) & 1;
      const int y0 = cur.b * BR;
      const int rows = min(BR, H - y0);
      if (wave == 4) ASR_BTR(1, 1, it - i0, 0);
      barrier_vm(0);  // this wave's x rows of band it landed
      if (wave == 4) ASR_BTR(1, 1, it - i0, 1);
#pragma unroll
      for (int q = 0; q < 2; ++q)
        if (fold && fp + q < fpe) fv[q] = *(const f32x4*)(pslabs + foff + (unsigned)q * ES);
      const bool more = it + 1 < i1;
      const int orow = more ? own_row(nxt.n == cur.n) : -1;
      unsigned mwv = 0u;
      // the next band's DMA pieces of this wave: own dy row (waves 0-3, or 0-5 when
      // the next band starts an image), x rows (waves 4-7; rows 2.. when it
      // continues this band's image); the first kBwd3Dma0 pieces issued here, the
      // rest after the band's MFMAs (below; the per-row interleave among the MFMAs
      // went with the round-5 cleanup d41213d, and this per-block path's speed was
      // not re-measured: the networks run the stacked kernels)
      if constexpr (EULER) {
        if (orow >= 0) mwv = bwd2_mask_word<C, W>(mask, nxt.n, nxt.b * BR, orow, H, lane);
      }
      const int xr0 = nxt.n == cur.n ? 2 : 0;
      const int ndy = orow >= 0 ? IPR : 0;
      const int nx = (more && w8 >= 4) ? ((BR + 2 - xr0) * IPR - (w8 - 4) + 3) / 4 : 0;
      const int npc = ndy + nx;
      int ipc = 0;
      auto piece = [&]() {
        if (ipc < ndy) {
          dma_row_instr<C, W>(dy, lds + L::DY + (buf ^ 1) * L::TILE + orow * L::ROWB, nxt.n, nxt.b * BR - 1 + orow,
                              ipc, H, loff);
        } else {
          dma_row_instr<C, W>(x, lds + L::X + (buf ^ 1) * L::TILE + xr0 * L::ROWB, nxt.n, nxt.b * BR - 1 + xr0,
                              (w8 - 4) + 4 * (ipc - ndy), H, loff);
        }
        ++ipc;
      };
      while (ipc < npc && ipc < kBwd3Dma0) piece();
      bf16x8 Bf[2], Ar[3];
      if (wave == 4) ASR_BTR(1, 1, it - i0, 2);
      // A fragments two m-tiles ahead (ring of 3), as in the round-1 v2 backward
      auto mfma_band = [&](auto bo) {
        constexpr int BO = decltype(bo)::value;
        Ar[0] = tr_pair_px<BO>(offA[0]);
        static_for<0, BR>([&](auto rc) {
          constexpr int r = decltype(rc)::value, RO_ = BO + r * L::ROWB;
          __builtin_amdgcn_sched_barrier(0);  // no hoisting of later rows' reads (register pressure)
          if (r < rows) {
            const bool mr = r + 1 < rows;
#pragma unroll
            for (int oi = 0; oi < 2; ++oi) Bf[oi] = tr_pair_px<RO_>(offB[oi]);
            Ar[1] = tr_pair_px<RO_>(offA[1]);
            static_for<0, MTW>([&](auto mc) {
              constexpr int mi = decltype(mc)::value;
              if constexpr (mi + 2 < MTW) Ar[(mi + 2) % 3] = tr_pair_px<RO_>(offA[mi + 2]);
              else if constexpr (mi + 2 == MTW && r + 1 < BR) {
                if (mr) Ar[0] = tr_pair_px<RO_ + L::ROWB>(offA[0]);  // MTW % 3 == 0: slot 0 again
              }
#pragma unroll
              for (int oi = 0; oi < 2; ++oi)
                acc[mi][oi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ar[mi % 3], Bf[oi], acc[mi][oi], 0, 0, 0);
            });
            if (dbw) {
#pragma unroll
              for (int oi = 0; oi < 2; ++oi)
                accb[oi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, Bf[oi], accb[oi], 0, 0, 0);
            }
          }
        });
      };
      if (it > i0) {  // the offsets follow the buffer (in place: no second register set)
        const unsigned dlt = buf ? (unsigned)L::TILE : (unsigned)-L::TILE;
#pragma unroll
        for (int mi = 0; mi < MTW; ++mi) offA[mi] += dlt;
#pragma unroll
        for (int oi = 0; oi < 2; ++oi) offB[oi] += dlt;
      }
      mfma_band(std::integral_constant<int, 0>{});
      while (ipc < npc) piece();
      if (more) {
        vm_wait(0);  // own dy row and mask dwords of band it+1 (x DMA and fold loads too: long landed)
        convert_own(orow, buf ^ 1, mwv);
      }
      if (wave == 4) ASR_BTR(1, 1, it - i0, 3);
      // halo rows of a band that continues this band's image: dz rows BR, BR+1
      // -> 0, 1 (masked), x rows BR, BR+1 -> 0, 1, dy row BR+1 -> 1; 5 x 256
      // chunks over the 512 wgrad threads
      if (it + 1 < i1 && nxt.n == cur.n) {
        const unsigned base = lds_u32(lds);
        const int nbf = buf ^ 1;
        u32x4 cv[3];
        unsigned dst[3];
        int nc = 0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int c = ft + 512 * k;
          if (c < 5 * 256) {
            const int which = c >> 8;
            const unsigned o = (unsigned)((c & 255) + NQ) * 16u;
            const unsigned sreg = which < 2 ? L::DZ : which < 4 ? L::X : L::DY;
            const int srow = which == 4 ? BR + 1 : BR + (which & 1);
            const int drow = which == 4 ? 1 : (which & 1);
            cv[k] = lds_rd128(base + sreg + buf * L::TILE + srow * L::ROWB + o);
            dst[k] = base + sreg + nbf * L::TILE + drow * L::ROWB + o;
            nc = k + 1;
          }
        }
        lgkm_wait<0>();
#pragma unroll
        for (int k = 0; k < 3; ++k)
          if (k < nc) lds_wr128(dst[k], cv[k]);
      }
#pragma unroll
      for (int q = 0; q < 2; ++q)
        if (fold && fp < fpe) {
          facc += fv[q];
          ++fp;
          foff += ES;
        }
      if (wave == 4) ASR_BTR(1, 1, it - i0, 4);
    }
    barrier_vm(0);  // all items consumed: LDS reusable
    if (dbw && g == 0) {
      float* dbl = (float*)lds + 12288;  // [C]
#pragma unroll
      for (int oi = 0; oi < 2; ++oi) dbl[16 * (oq + oi) + lx] = hs * accb[oi][0];
    }
    constexpr int MC = XT ? 3 : MTW;
#pragma unroll
    for (int m0 = 0; m0 < MTW; m0 += MC) {
      float prev[XT ? MC : 1][2][4];
      if constexpr (XT) {
#pragma unroll
        for (int mi = 0; mi < MC; ++mi)
#pragma unroll
          for (int oi = 0; oi < 2; ++oi)
#pragma unroll
            for (int e = 0; e < 4; ++e)
              prev[mi][oi][e] = slab[(long)(16 * (tg * MTW + m0 + mi) + 4 * g + e) * C + 16 * (oq + oi) + lx];
      }
#pragma unroll
      for (int mi = 0; mi < MC; ++mi)
#pragma unroll
        for (int oi = 0; oi < 2; ++oi)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int m = 16 * (tg * MTW + m0 + mi) + 4 * g + e;
            float v = hs * acc[m0 + mi][oi][e];
            if constexpr (XT) v += prev[mi][oi][e];
            slab[(long)m * C + 16 * (oq + oi) + lx] = v;
          }
    }
  }
  __syncthreads();
  if (tid < C) {
    const float* dbl = (const float*)lds + 12288;
    float s = dbl[tid];
    if constexpr (XT) s += slab[9 * C * C + tid];
    slab[9 * C * C + tid] = s;
  }
  if (fold) {  // slabs the bands did not cover (a WG with fewer than 16 bands)
    for (; fp < fpe; ++fp, foff += ES) facc += *(const f32x4*)(pslabs + foff);
    *(f32x4*)(pgrp + (long)fg * ES + (foff - (unsigned)fpe * ES)) = facc;
  }
  ASR_BCLK(1, 1);
}

// ===========================================================================
// Stack backward (C=64, W=32, BR=4, Euler): the backward of all L blocks in
// ONE launch, k_bwd3's band protocol and roles on (block, image, band) items,
// blocks last to first.  A workgroup owns whole images (as k_fwd3_stack), so
// block l-1 of an image reads only the dx this workgroup wrote for block l
// (ping-pong buffers dbuf[0/1]: block L-1 reads dbuf[0]); the only exchange
// between workgroups is the weight-gradient reduction:
//   * at the end of its items of block l, every wgrad wave stores its dW
//     tiles as sc1 (write-through) 16-B stores in the tile-major slab layout
//       slab[((mt * 4 + ot) * 64 + lane) * 4 + e] = dW[16 mt + 4 (lane>>4) + e][16 ot + (lane&15)]
//     (db after the 9C^2 block); the next band barrier drains them (vmcnt(0))
//     and one lane adds 1 to done[l] (relaxed, agent scope: the Guideline-16
//     write-through publish);
//   * pass 1 of block l's reduction (32-slab group sums, as k_bwd3's fold) is
//     folded into this workgroup's bands of block l-2: one lane polls done[l]
//     == gridDim.x before the first of them and fences acquire at agent scope,
//     and the band barrier orders that before every slab load.  Blocks below
//     lfold (>= 2; L when a workgroup would own more than 512 chunks of the
//     group rows, one per wgrad thread) are reduced after the launch.
//   * the poll is bounded (kStackSpinLimit sleeps, ~1-2 ms): a missed hand-off
//     costs speed, never correctness.  A workgroup whose wait runs out sets
//     skipf[l] (its share of block l's group rows may be built from slabs not
//     yet published), counts the event in g_stack_degraded (asr_stack_status),
//     and stops waiting for the rest of the launch (a word in LDS): every later
//     block it folds is flagged too.  After the launch, stack_bwd_reduce_rest
//     recomputes the group rows of every flagged block from its slabs, which
//     are all published by then (same stream), before the projection reads them.
// Co-residency of the grid (one 768-thread workgroup per CU, grid <= CUs; the
// stacked path is used only when the occupancy query keeps one resident per
// CU) is therefore a speed matter: a grid that is not (another kernel or
// process on the device) degrades to the post-launch reduction of the blocks
// whose wait ran out.  At the switch to block l-1 the dgrad waves load its W
// after their last conv of block l; block 0 applies the stem's relu' to dx
// when ro0 (k_bwd3<..., RO>).
// ===========================================================================
typedef __attribute__((address_space(1))) unsigned gu32;  // global agent-scope words (never flat)
// bound of the stacked backward's slab wait, in polls of one relaxed L2 load
// + s_sleep 2 (~1-2 ms: about one whole launch, far above the skew between
// resident workgroups, which stay within a block of each other).  A
// compile-time constant: a run-time bound cost the kernel a spilled register
// (tests/test_isa.py)
constexpr unsigned kStackSpinLimit = 1u << 13;
// waits of k_bwd3_stack workgroups that ran out since the last reset
// (asr_stack_status): each one means a slower launch (post-launch reduction of
// the flagged blocks), not a wrong gradient
__device__ unsigned g_stack_degraded = 0u;
typedef __attribute__((address_space(1))) float gf32;

// Pair-local weight-gradient tiling of k_bwd3_stack<..., PAIR> (C = 64, an
// antisymmetric operator: W[8-t][o][i] = -W[t][i][o] for tap t = 3ky+kx,
// …3By3.py:115-141, 277-293).  Every theta then pulls back
// D(t,i,o) = dW[t][i][o] - dW[8-t][o][i] (one entry, a sign), so the slab
// stores D, not dW: 74 16x16 tiles instead of 144 (half the publish burst
// and half the fold's reads).  Wave w8 = 2p + h of the 8 wgrad waves owns tap
// pair (p, 8-p) for input tiles a = 0..3 and output tiles b in {2h, 2h+1}:
// X = dW[p] tiles (A = x(p, a), B = dz(b)) and the transposed dW[8-p] tiles
// (A = dz(a), B = x(8-p, b): the same fragments in the other operand slot
// give the transpose), D = X - Y^T in registers; plus 2 MFMAs of tap 4:
// waves p < 3 one cross pair (a', b') of tiles (D likewise), waves p = 3 the
// two self tiles of their b-set (raw, and transposed for the odd one; the
// projection forms X - X^T there).  perm(0..3) orders the tiles a wave walks
// (its b-set first) so that every accumulator and register index is
// compile-time: acc[a][b] / acc[4+a][b] hold tiles (perm(a), perm(b)).
using PairSlab = PairSlabLayout;
constexpr int cmin(int a, int b) { return a < b ? a : b; }
// the pipelined pair wgrad (k_bwd3_stack): the last of a row's 12 fragments MFMA group g uses
constexpr int pf_last(int g) { return g == 0 ? 2 : g == 1 ? 3 : g == 2 ? 5 : g + 3; }  // (asr_common.h: the layout and the projection's pair_encode)
struct PairRole {
  // one wave-uniform word (the wgrad role sits at the SGPR limit): bits 0-7 perm(0..3),
  // 8-9 t, 10 self, 11 (s1 == 2), 12-14 k4
  unsigned w;
  __device__ __forceinline__ explicit PairRole(int w8) {
    const int t = w8 >> 1, h = w8 & 1, self = t == 3;
    // tap-4 cross pair k4 = (a', b') with b' in the wave's b-set {2h, 2h+1}
    const int k4 = 3 * h + t;
    const int ap = pair_tap4_a(k4), bp = pair_tap4_b(k4);
    const int b0 = self ? 2 * h : bp, b1 = (4 * h + 1) - b0;  // the b-set, b0 first
    // perm(2): a' when a' is outside the b-set (the tap-4 transposed product reads dz(perm(s1)))
    const int o0 = h ? 0 : 2, o1 = h ? 1 : 3;  // the two tiles outside the b-set
    const bool ain = !self && (ap >> 1) == h;
    const int p2 = (!self && !ain) ? ap : o0, p3 = (p2 == o0) ? o1 : o0;
    const int s2 = (self || ain) ? 0 : 1;
    w = (unsigned)(b0 | (b1 << 2) | (p2 << 4) | (p3 << 6) | (t << 8) | (self << 10) | (s2 << 11) | (k4 << 12));
  }
  __device__ __forceinline__ int perm(int k) const { return (w >> (2 * k)) & 3; }
  __device__ __forceinline__ int t() const { return (w >> 8) & 3; }
  __device__ __forceinline__ bool self() const { return (w >> 10) & 1; }
  __device__ __forceinline__ bool s1_is_2() const { return (w >> 11) & 1; }
  __device__ __forceinline__ int k4() const { return (int)(w >> 12) & 7; }
  // tap-4 fragments: x(4, u0) (phase 2, with dz(perm 0)), x(4, v1) (phase 1, with dz(perm s1))
  __device__ __forceinline__ int u0() const { return self() ? perm(0) : pair_tap4_a(k4()); }
  __device__ __forceinline__ int v1() const { return self() ? perm(1) : pair_tap4_b(k4()); }
  // LDS address bits of tile perm(k) relative to tile 0 (wave-uniform: one v_xor per read)
  __device__ __forceinline__ unsigned sh(int k) const { return (unsigned)perm(k) << 5; }
  // slab tile of acc[a][b] (D of tap t, input tile perm(a), output tile perm(b))
  __device__ __forceinline__ int tile(int a, int b) const { return t() * 16 + perm(a) * 4 + perm(b); }
};

// RK2 (config 5): items walk 2L stages, per block l its second stage first
// (dy = dL/dx_{l+1}, x = xmid_l, mask2, h, no +dy residual: out g = A^T dz2 into
// gbuf) then its first (dy = g, x = x_l, mask1, h/2, plus the extra term
// dL/dx_{l+1} by 16-B global loads: out dx_l).  Both stages accumulate one dW:
// at the stage switch acc *= 2 (exact), and the block's slab is (h/2) acc.
template <int C, int W, int BR, bool RK2 = false, bool PAIR = false>
__global__ __launch_bounds__(768, 1) void k_bwd3_stack(bf16* __restrict__ dbuf0, bf16* __restrict__ dbuf1,
                                                       const bf16* __restrict__ xs, long x_stride,
                                                       const uint8_t* __restrict__ masks, long mask_stride,
                                                       const bf16* __restrict__ wpack, long w_stride, float h,
                                                       float two_gamma, int N, int H, int L, int ro0,
                                                       float* __restrict__ slabs, long slab_stride,
                                                       float* __restrict__ grp, long grp_stride,
                                                       unsigned* __restrict__ done, unsigned* __restrict__ skipf,
                                                       int lfold, const bf16* __restrict__ xm = nullptr,
                                                       const uint8_t* __restrict__ masks2 = nullptr,
                                                       bf16* __restrict__ gbuf = nullptr,
                                                       const bf16* __restrict__ gtop = nullptr) {
  using G = Geo<C>;
  using LL = Bwd2Lds<C, W, BR>;
  using BD = Band<C, W, BR>;
  constexpr int TW = W + 2, OT = G::OT, MTW = G::MTW, IPR = W / G::PPI, NQ = G::NQ;
  static_assert(C == 64 && W == 32 && BR == 4 && MTW == 9 && OT == 4, "v3 backward geometry");
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, lx = lane & 15;

  for (int b = 0; b < 2; ++b) {
    zero_halo_cols<C, W>(lds + LL::DY + b * LL::TILE, BR + 2, tid, 768);
    zero_halo_cols<C, W>(lds + LL::X + b * LL::TILE, BR + 2, tid, 768);
    zero_halo_cols<C, W>(lds + LL::DZ + b * LL::TILE, BR + 2, tid, 768);
  }
  {
    unsigned* tab = (unsigned*)(lds + LL::MTAB);
    for (int i = tid; i < 1024; i += 768) {
      const unsigned m = (unsigned)i >> 2, d = (unsigned)i & 3;
      tab[i] = (((m >> (2 * d)) & 1u) ? 0xffffu : 0u) | (((m >> (2 * d + 1)) & 1u) ? 0xffff0000u : 0u);
    }
  }
  // the LDS byte address of the allocation, taken here (uniform code): casting in the dgrad
  // role's code made hipcc (ROCm 7.2) emit the cast's null check as an illegal VALU compare
  const unsigned lds0 = lds_u32(lds);
  unsigned* late = (unsigned*)(lds + LL::TOTAL);  // a slab wait of this workgroup ran out: stop waiting
  if (tid == 0) *late = 0u;
  const int n0 = (int)((long)blockIdx.x * N / gridDim.x), n1 = (int)((long)(blockIdx.x + 1) * N / gridDim.x);
  // cursor index l is a STAGE: the block itself (Euler) or 2*block + (1: second RK2 stage, 0: first)
  constexpr int SPB = RK2 ? 2 : 1;
  const int nb = (H + BR - 1) / BR, per = (n1 - n0) * nb, total = SPB * L * per;
  const unsigned loff = (unsigned)dma_lane_off<C, W>(lane) * 2u;
  auto blk_of = [&](int st) { return RK2 ? st >> 1 : st; };
  auto s1_of = [&](int st) { return RK2 && !(st & 1); };  // first RK2 stage: h/2, extra term
  // block l reads dL/dx_{l+1} from dbuf[(L-1-l) & 1] and writes dL/dx_l to the other one
  auto din_of = [&](int l) -> bf16* { return ((L - 1 - l) & 1) ? dbuf1 : dbuf0; };
  auto dout_of = [&](int l) -> bf16* { return ((L - 1 - l) & 1) ? dbuf0 : dbuf1; };
  auto dy_of = [&](int st) -> bf16* {
    if constexpr (RK2) return (st & 1) ? din_of(st >> 1) : gbuf;
    else return din_of(st);
  };
  auto dx_of = [&](int st) -> bf16* {
    if constexpr (RK2) return (st & 1) ? gbuf : dout_of(st >> 1);
    else return dout_of(st);
  };
  auto x_of = [&](int st) -> const bf16* {
    if constexpr (RK2) return ((st & 1) ? xm : xs) + (long)(st >> 1) * x_stride;
    else return xs + (long)st * x_stride;
  };
  auto mask_of = [&](int st) -> const uint8_t* {
    if constexpr (RK2) return ((st & 1) ? masks2 : masks) + (long)(st >> 1) * mask_stride;
    else return masks + (long)st * mask_stride;
  };
  // (block, image, band) cursor, blocks last to first
  struct Cur {
    int l, n, b;
  };
  auto adv = [&](Cur& c) {
    if (++c.b == nb) {
      c.b = 0;
      if (++c.n == n1) {
        c.n = n0;
        --c.l;
      }
    }
  };
  __syncthreads();
  if (n0 >= n1) return;  // (uniform per workgroup: never with grid <= N)
  ASR_BCLK(1, 0);

  constexpr int ES = PAIR ? PairSlab::ES : 9 * C * C + C, ECH = ES / 4;
  if (wave < 4) {
    // ---------------- dgrad waves ----------------
    const int ot = wave;
    // W by untracked loads, here and at each block switch: the next item's
    // barrier_vm retires them (a tracked reload made hipcc wait vmcnt(0) before
    // every band's first MFMA, i.e. for the previous band's dx stores)
    bf16x8 A[G::KS] = {};
    load_A1_untracked<C>(wpack + (long)(L - 1) * w_stride, ot, lane, A);
    unsigned lo[3 * BD::NCB];
    band_lane_offsets<C, W, BR>(g, lx, lo);
    const int px = lx + 16 * (g & 1), cg = 2 * ot + (g >> 1);
    const unsigned lch = (unsigned)toff<C>(1, px + 1, cg, TW);
    const unsigned ldx = (unsigned)(px * C + 8 * cg) * 2u;
    int nst = 0;
    Cur cur{SPB * L - 1, n0, 0};
    for (int it = 0; it < total; ++it) {
      const int buf = it & 1;
      const int n = cur.n, y0 = cur.b * BR, l = cur.l;
      const int rows = min(BR, H - y0);
      if (wave == 0) ASR_BTR(1, 0, it, 0);
      const bool sw_ = !RK2 && cur.b == 0 && n == n0;  // (trace build: the first band of block l)
      if (wave == 0 && sw_) ASR_BSW(l, 3, false);
      barrier_vm_usual<BR>(nst);  // item it staged everywhere; item it-1 fully consumed
      if (wave == 0) ASR_BTR(1, 0, it, 1);
      if (wave == 0 && sw_) ASR_BSW(l, 4, false);
      const unsigned dzt = lds_u32(lds + LL::DZ + buf * LL::TILE), dyt = lds_u32(lds + LL::DY + buf * LL::TILE);
      const unsigned xt = lds_u32(lds + LL::X + buf * LL::TILE);
      const bool s1 = s1_of(l);
      const float hs = s1 ? 0.5f * h : h, hs2g = hs * two_gamma;
      // RK2 first stage: the extra dx term dL/dx_{l+1} of the band's rows (in flight during the conv)
      u32x4 exv[RK2 ? BR : 1];
      if (RK2 && s1) {
        const bf16* eb = din_of(blk_of(l)) + ((long)n * H + y0) * W * C;
#pragma unroll
        for (int r = 0; r < (RK2 ? BR : 1); ++r)
          exv[r] = *(const u32x4*)((const unsigned char*)(eb + (long)min(r, rows - 1) * W * C) + ldx);
      }
      f32x4 acc[BR][2];
#pragma unroll
      for (int r = 0; r < BR; ++r) acc[r][0] = acc[r][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      conv_band<C, W, BR>(dzt, lo, A, acc);
      if (wave == 0) ASR_BTR(1, 0, it, 2);
      const bool last_of_stage = cur.b == nb - 1 && n == n1 - 1;
      if (last_of_stage && blk_of(l) > 0 && (!RK2 || s1))
        load_A1_untracked<C>(wpack + (long)(blk_of(l) - 1) * w_stride, ot, lane, A);
      bf16* drow = dx_of(l) + ((long)n * H + y0) * W * C;
      // dx rows as buffer stores (uniform base, the lane's 32-bit offset, the row as the scalar offset)
      const auto drs = __builtin_amdgcn_make_buffer_rsrc((void*)(RK2 ? nullptr : drow), 0, BR * W * C * 2, 0x00020000);
      int nld = 0;
      auto epilogue = [&](auto g2c, auto roc, auto kc) {
        // KIND 0: Euler (+dy), 1: second RK2 stage (no +dy), 2: first RK2 stage (+dy +extra)
        constexpr bool G2 = decltype(g2c)::value, RO = decltype(roc)::value;
        constexpr int KIND = decltype(kc)::value;
        constexpr bool RDY = KIND != 1;
        constexpr int NR = (RDY ? 1 : 0) + (G2 ? 1 : 0) + (RO ? 1 : 0);  // LDS reads per row
        u32x4 dyw[2], dzw[2], xw[2];
        auto issue = [&](int r, int sl) {
          const unsigned co = lch + (unsigned)(r * LL::ROWB);
          if constexpr (RDY) dyw[sl] = lds_rd128(dyt + co);
          if constexpr (G2) dzw[sl] = lds_rd128(dzt + co);
          if constexpr (RO) xw[sl] = lds_rd128(xt + co);
        };
        // the reads run on a compile-time schedule, each retired before the row guard,
        // so no branch sits between a read and the wait that retires it: with the
        // reads inside the guard hipcc merged a read's register at the join with a copy
        // placed before that wait (stale dy rows under LDS contention, tools/asm_lds_audit.py)
        if constexpr (NR > 0) issue(0, 0);
        static_for<0, BR>([&](auto rc) {
          constexpr int r = decltype(rc)::value, sl = r & 1;
          if constexpr (NR > 0) {
            if constexpr (r + 1 < BR) {
              issue(r + 1, sl ^ 1);
              lgkm_wait<NR>();
            } else {
              lgkm_wait<0>();
            }
          }
          if (r < rows) {
            float z[8];
            regroup(acc[r][0], acc[r][1], z);
            u32x4 ow;
#pragma unroll
            for (int d = 0; d < 4; ++d) {
              float r0 = 0.f, r1 = 0.f;
              if constexpr (RDY) r0 = lo_f(dyw[sl][d]), r1 = hi_f(dyw[sl][d]);
              if constexpr (KIND == 2) {
                r0 += lo_f(exv[RK2 ? r : 0][d]);
                r1 += hi_f(exv[RK2 ? r : 0][d]);
              }
              float v0 = fmaf(-hs, z[2 * d], r0);
              float v1 = fmaf(-hs, z[2 * d + 1], r1);
              if constexpr (G2) {
                v0 = fmaf(hs2g, lo_f(dzw[sl][d]), v0);
                v1 = fmaf(hs2g, hi_f(dzw[sl][d]), v1);
              }
              ow[d] = pk_bf16(v0, v1);
              if constexpr (RO) {
                const unsigned xd = xw[sl][d];
                ow[d] &= ((int)(short)(xd & 0xffffu) > 0 ? 0xffffu : 0u) | ((int)xd > 0xffff ? 0xffff0000u : 0u);
              }
            }
            if constexpr (RK2)  // (its dgrad role has no SGPRs to spare for the descriptor)
              *(u32x4*)((unsigned char*)(drow + (long)r * W * C) + ldx) = ow;
            else
              __builtin_amdgcn_raw_buffer_store_b128(ow, drs, (int)ldx, r * W * C * 2, 0);
            ++nld;
          }
        });
      };
      using T_ = std::true_type;
      using F_ = std::false_type;
      using K0 = std::integral_constant<int, 0>;
      using K1 = std::integral_constant<int, 1>;
      using K2 = std::integral_constant<int, 2>;
      const bool g2 = hs2g != 0.f;
      if constexpr (RK2) {
        if (s1) {
          if (g2) epilogue(T_{}, F_{}, K2{});
          else epilogue(F_{}, F_{}, K2{});
        } else {
          if (g2) epilogue(T_{}, F_{}, K1{});
          else epilogue(F_{}, F_{}, K1{});
        }
      } else {
        const bool ro = ro0 && l == 0;
        if (ro) {
          if (g2) epilogue(T_{}, T_{}, K0{});
          else epilogue(F_{}, T_{}, K0{});
        } else {
          if (g2) epilogue(T_{}, F_{}, K0{});
          else epilogue(F_{}, F_{}, K0{});
        }
      }
      nst = nld;
      if (wave == 0) ASR_BTR(1, 0, it, 3);
      if (!RK2 && cur.b + 1 < nb) {  // (RK2: the wgrad waves copy them; its dgrad role has no registers to spare)
        // the next item continues this image: its tile rows 0, 1 are this band's rows BR, BR+1
        // (dz, x; dy row 1 only), copied here, where the dgrad waves would otherwise wait at
        // the band barrier for the wgrad waves.  Rows BR, BR+1 of this item's tiles were
        // complete at its barrier, and no wave touches rows 0, 1 of the other buffer before
        // the next one (its DMAs and the convert fill rows 2..).  Compiler-visible LDS
        // accesses: the epilogue's asm reads were retired by its last lgkm_wait<0>, and these
        // waves have no LDS-DMA in flight
        const unsigned base = lds0;
        const int nbf = buf ^ 1;
#pragma unroll
        for (int k = 0; k < 5; ++k) {
          const int c = tid + 256 * k;  // 5 x 256 16-B chunks: dz rows, x rows, dy row
          const unsigned o = (unsigned)((c & 255) + NQ) * 16u;
          const unsigned sreg = k < 2 ? LL::DZ : k < 4 ? LL::X : LL::DY;
          const int srow = k == 4 ? BR + 1 : BR + (k & 1);
          const int drow = k == 4 ? 1 : (k & 1);
          lds_st128(base + sreg + nbf * LL::TILE + drow * LL::ROWB + o,
                    lds_ld128(base + sreg + buf * LL::TILE + srow * LL::ROWB + o));
        }
      }
      if (wave == 0) ASR_BTR(1, 0, it, 4);
      adv(cur);
    }
    barrier_vm(0);  // matches the wgrad waves' end-of-loop barrier
  } else {
    // ---------------- wgrad waves ----------------
    const int w8 = __builtin_amdgcn_readfirstlane(wave) - 4;
    const int tg = w8 >> 1, oq = 2 * (w8 & 1);
    const int tq = lx >> 2, tp = lx & 3;
    const int ft = tid - 256;
    f32x4 acc[MTW][2];
#pragma unroll
    for (int mi = 0; mi < MTW; ++mi) acc[mi][0] = acc[mi][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    // operand addresses: the full-dW tiling (PAIR false) reads 9 x fragments (offA) and 2 dz
    // fragments (offB) per row; the pair-local tiling (PairRole) 8 x and 4 dz fragments
    constexpr int NOA = PAIR ? 5 : MTW, NOB = PAIR ? 1 : 2;
    unsigned offA[NOA], offB[NOB];  // pixel tile 1 sits 16 px = 2 KiB on (swizzle period 8 px)
    const PairRole pr(w8);
    {
      const unsigned xb0 = lds_u32(lds + LL::X), zb0 = lds_u32(lds + LL::DZ);
      const int pb = 4 * g + tq;
      auto xoff = [&](int tap, int itile) {
        const int ky = tap / 3, kx = tap % 3, q = 2 * itile + (tp >> 1);
        return xb0 + (unsigned)(toff<C>(ky, pb + kx, q, TW) + 8 * (tp & 1));
      };
      auto zoff = [&](int otile) {
        return zb0 + (unsigned)(toff<C>(1, pb + 1, 2 * otile + (tp >> 1), TW) + 8 * (tp & 1));
      };
      if constexpr (PAIR) {
        // offA: x(t, tile 0), x(8-t, perm[0]), x(8-t, perm[1]), x(4, u0), x(4, v1); offB: dz(tile 0).
        // A 16-channel tile's fragment address differs from tile 0's only in address bits 5-6
        // (the chunk index 2*tile + h, XOR-swizzled by the column: (tile ^ (col&7)>>1) << 5; the
        // buffer bases and the tile-buffer step keep those bits clear), so x(t, a) and dz(a) are
        // read at offA[0] ^ (a << 5), offB[0] ^ (a << 5): one register each instead of four
        offA[0] = xoff(pr.t(), 0);
        offA[1] = xoff(8 - pr.t(), pr.perm(0));
        offA[2] = xoff(8 - pr.t(), pr.perm(1));
        offA[3] = xoff(4, pr.u0());
        offA[4] = xoff(4, pr.v1());
        offB[0] = zoff(0);
      } else {
#pragma unroll
        for (int mi = 0; mi < MTW; ++mi) {
          const int mt = tg * MTW + mi;
          offA[mi] = xoff((16 * mt) / C, ((16 * mt) % C) / 16);
        }
#pragma unroll
        for (int oi = 0; oi < 2; ++oi) offB[oi] = zoff(oq + oi);
      }
      // opaque to the compiler: kept in VGPRs, not recomputed per band
#pragma unroll
      for (int k = 0; k < NOA; ++k) asm volatile("" : "+v"(offA[k]));
#pragma unroll
      for (int k = 0; k < NOB; ++k) asm volatile("" : "+v"(offB[k]));
    }
    auto own_row = [&](bool reuse) { return reuse ? (w8 < 4 ? 2 + w8 : -1) : (w8 < 6 ? w8 : -1); };
    // gtop (Euler): the top block's dy = dL/dx_L is the GAP gradient, one row per image constant over the
    // pixels (tfkeras_resnets.py:595-597); its tile rows are written from that row (zeros outside the
    // image, as the DMA's zero page) instead of read from a full tensor
    auto synth = [&](const Cur& c) { return !RK2 && gtop != nullptr && c.l == L - 1; };
    auto synth_row = [&](const Cur& c, int row, int nbuf) {
      const int gy = c.b * BR - 1 + row, q = lane & 7, p0 = lane >> 3;
      u32x4 v = {0u, 0u, 0u, 0u};
      if ((unsigned)gy < (unsigned)H) {  // (buffer load: a 32-bit lane offset, no 64-bit per-lane pointer kept live)
        const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(gtop + (long)c.n * C), 0, C * 2, 0x00020000);
        v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * q, 0, 0));
      }
      const unsigned rb = lds_u32(lds + LL::DY + nbuf * LL::TILE + row * LL::ROWB);
#pragma unroll
      for (int k = 0; k < W / 8; ++k) lds_st128(rb + (unsigned)toff<C>(0, p0 + 8 * k + 1, q, TW), v);
    };
    auto stage_own = [&](const Cur& c, int row, int nbuf, unsigned& mwv) {
      if (row < 0) return;
      mwv = bwd2_mask_word<C, W>(mask_of(c.l), c.n, c.b * BR, row, H, lane);
      if (synth(c)) {
        synth_row(c, row, nbuf);
        return;
      }
      for (int j = 0; j < IPR; ++j)
        dma_row_instr_at<C, W>(dy_of(c.l), lds0 + (unsigned)(LL::DY + nbuf * LL::TILE + row * LL::ROWB), c.n, c.b * BR - 1 + row, j,
                            H, loff);
    };
    auto convert_own = [&](int row, int nbuf, unsigned mwv) {
      if (row < 0) return;
      const unsigned base = lds_u32(lds);
      const int cpx = lane & 31, hh = lane >> 5;
#pragma unroll
      for (int jj = 0; jj < 4; jj += 2) {
        u32x4 v[2], mt[2];
        unsigned off[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          off[j] = (unsigned)toff<C>(row, cpx + 1, 4 * hh + jj + j, TW) + (unsigned)(nbuf * LL::TILE);
          v[j] = lds_ld128(base + LL::DY + off[j]);
          mt[j] = lds_ld128(base + LL::MTAB + __builtin_amdgcn_ubfe(mwv, 8 * (jj + j), 8) * 16);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          u32x4 z = v[j];
          z &= mt[j];
          lds_st128(base + LL::DZ + off[j], z);
        }
      }
    };
    bf16x8 ones;
#pragma unroll
    for (int i = 0; i < 8; ++i) ones[i] = (bf16)1.0f;
    f32x4 accb[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    const bool dbw = PAIR ? pr.self() : tg == 3;
    // fold state (pass 1 of block l+2's reduction while on block l)
    const long fT = (long)((gridDim.x + 31) / 32) * ECH;
    const long fc0 = (long)blockIdx.x * fT / gridDim.x, fc1 = (long)(blockIdx.x + 1) * fT / gridDim.x;
    const bool fmine = ft >= 0 && fc0 + ft < fc1;
    const int fg = fmine ? (int)((fc0 + ft) / ECH) : 0;
    const int fpe = min((int)gridDim.x, 32 * fg + 32);
    const unsigned fch = fmine ? (unsigned)((fc0 + ft) % ECH) * 4 : 0u;
    bool fold = false;
    int fp = 0;
    unsigned foff = 0u;
    const float* pslabs = slabs;
    f32x4 facc = {0.f, 0.f, 0.f, 0.f}, fv[2];
    auto fold_begin = [&](int l) {  // block l's slabs (published: done[l] == grid, acquired)
      fold = fmine;
      fp = 32 * fg;
      foff = (unsigned)fp * ES + fch;
      pslabs = slabs + (long)l * slab_stride;
      facc = f32x4{0.f, 0.f, 0.f, 0.f};
    };
    auto fold_end = [&](int l) {
      if (fold) {
        for (; fp < fpe; ++fp, foff += ES) facc += *(const f32x4*)(pslabs + foff);
        // (the group row's offset from live values: foff - fpe*ES is this thread's chunk)
        *(f32x4*)(grp + (long)l * grp_stride + ((unsigned)fg * ES + (foff - (unsigned)fpe * ES))) = facc;
      }
      fold = false;
    };
    const float hsb = RK2 ? 0.5f * h : h;  // the slab scale (RK2: acc doubled at the stage switch)
    {  // prologue: own dy rows and x rows of item 0, its dz converted
      const Cur c0{SPB * L - 1, n0, 0};
      unsigned mw0 = 0u;
      const int row0 = own_row(false);
      stage_own(c0, row0, 0, mw0);
      for (int j = w8; j < (BR + 2) * IPR; j += 8)
        dma_row_instr_at<C, W>(x_of(c0.l), lds0 + (unsigned)LL::X, c0.n, c0.b * BR - 1, j, H, loff);
      vm_wait(0);
      convert_own(row0, 0, mw0);
    }
    Cur cur{SPB * L - 1, n0, 0}, nxt{SPB * L - 1, n0, 0};
    adv(nxt);
    for (int it = 0; it < total; ++it) {
      const int buf = it & 1;
      const int y0 = cur.b * BR, l = blk_of(cur.l);  // (l: the block)
      const int rows = min(BR, H - y0);
      const bool first_of_block = cur.b == 0 && cur.n == n0 && (!RK2 || (cur.l & 1));
      if (wave == 4) ASR_BTR(1, 1, it, 0);
      if (wave == 4 && first_of_block && !RK2) {
        ASR_BSW(l, 0, false);
        ASR_BSW(l, 5, true);
      }
      if (first_of_block && l + 2 < L && l + 2 >= lfold && w8 == 0 && lane == 0) {
        // block l+2's slabs: every workgroup published them (bounded poll); once a
        // wait of this workgroup ran out, every later block it folds is flagged
        // for the post-launch reduction instead (stack_bwd_reduce_rest)
        bool ran_out = *(volatile unsigned*)late != 0u;
        if (!ran_out) {
          unsigned spins = 0;
          while (__hip_atomic_load((gu32*)(done + l + 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gridDim.x) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins > kStackSpinLimit) {
              ran_out = true;
              *(volatile unsigned*)late = 1u;
              __hip_atomic_fetch_add((gu32*)&g_stack_degraded, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              break;
            }
          }
        }
        if (ran_out) __hip_atomic_store((gu32*)(skipf + l + 2), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      }
      if (wave == 4 && first_of_block && !RK2) ASR_BSW(l, 1, false);
      barrier_vm(0);  // this wave's x rows of item it landed (and its slab stores drained)
      if (wave == 4) ASR_BTR(1, 1, it, 1);
      if (wave == 4 && first_of_block && !RK2) {
        ASR_BSW(l, 2, false);
        ASR_BSW(l, 6, true);
      }
      if (first_of_block && l + 1 < L && l + 1 >= lfold && w8 == 0 && lane == 0)
        __hip_atomic_fetch_add((gu32*)(done + l + 1), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // published
      if (first_of_block && l + 2 < L && l + 2 >= lfold) fold_begin(l + 2);
#pragma unroll
      for (int q = 0; q < 2; ++q)
        if (fold && fp + q < fpe) fv[q] = *(const f32x4*)(pslabs + foff + (unsigned)q * ES);
      const bool more = it + 1 < total;
      const bool cont = more && nxt.l == cur.l && nxt.n == cur.n;
      const int orow = more ? own_row(cont) : -1;
      unsigned mwv = 0u;
      if (orow >= 0) mwv = bwd2_mask_word<C, W>(mask_of(nxt.l), nxt.n, nxt.b * BR, orow, H, lane);
      const int xr0 = cont ? 2 : 0;
      const bool syn = orow >= 0 && synth(nxt);
      if (syn) synth_row(nxt, orow, buf ^ 1);
      // the next band's rows, each by one whole-row DMA (4 pieces on one address): the own dy
      // row, and x rows 2..5 on waves 4..7 when the next band continues this image (rows 0, 1
      // are the halo copy), else rows 0..5 with row r on wave (r + 6) & 7.  (Measured and not
      // kept: the x rows DMA'd by the dgrad waves before their conv, -1.8 %, r05c)
      if (orow >= 0 && !syn)
        dma_row_whole_at<C, W>(dy_of(nxt.l), lds0 + (unsigned)(LL::DY + (buf ^ 1) * LL::TILE + orow * LL::ROWB), nxt.n,
                               nxt.b * BR - 1 + orow, H, loff);
      if (more) {
        const int xrow = cont ? (w8 >= 4 ? w8 - 2 : -1) : (((w8 + 2) & 7) < BR + 2 ? ((w8 + 2) & 7) : -1);
        if (xrow >= 0)
          dma_row_whole_at<C, W>(x_of(nxt.l), lds0 + (unsigned)(LL::X + (buf ^ 1) * LL::TILE + xrow * LL::ROWB), nxt.n,
                                 nxt.b * BR - 1 + xrow, H, loff);
      }
      if (wave == 4) ASR_BTR(1, 1, it, 2);
      bf16x8 Bf[2], Ar[3];
      auto mfma_band_full = [&](auto bo) {
        constexpr int BO = decltype(bo)::value;
        Ar[0] = tr_pair_px<BO>(offA[0]);
        static_for<0, BR>([&](auto rc) {
          constexpr int r = decltype(rc)::value, RO_ = BO + r * LL::ROWB;
          __builtin_amdgcn_sched_barrier(0);
          if (r < rows) {
            const bool mr = r + 1 < rows;
#pragma unroll
            for (int oi = 0; oi < 2; ++oi) Bf[oi] = tr_pair_px<RO_>(offB[oi]);
            Ar[1] = tr_pair_px<RO_>(offA[1]);
            static_for<0, MTW>([&](auto mc) {
              constexpr int mi = decltype(mc)::value;
              if constexpr (mi + 2 < MTW) Ar[(mi + 2) % 3] = tr_pair_px<RO_>(offA[mi + 2]);
              else if constexpr (mi + 2 == MTW && r + 1 < BR) {
                if (mr) Ar[0] = tr_pair_px<RO_ + LL::ROWB>(offA[0]);
              }
#pragma unroll
              for (int oi = 0; oi < 2; ++oi)
                acc[mi][oi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ar[mi % 3], Bf[oi], acc[mi][oi], 0, 0, 0);
            });
            if (dbw) {
#pragma unroll
              for (int oi = 0; oi < 2; ++oi)
                accb[oi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, Bf[oi], accb[oi], 0, 0, 0);
            }
          }
        });
      };
      // pair-local tiling (PairRole): per row, phase 1 the transposed products of tap 8-t
      // (A = dz(perm[a]), B = -x(8-t, perm[b]): -dW[8-t]^T tiles) and the tap-4 partner's,
      // phase 2 the direct products of tap t (A = x(t, perm[a]), B = dz(perm[b])) and the
      // tap-4 tile, both into acc[a][b], which holds D = X - Y^T at the block's end.
      // The band's 4 x 12 operand fragments are one read stream, each read issued P = 3
      // fragments ahead of the MFMA group that first uses it, across the row boundaries
      // (the transposed reads are compiler-visible builtins: hipcc places their waits; a
      // version reading each row's fragments at the row's start ran its MFMA phase 0.5-0.6 k
      // cycles longer per band); row r's fragments in use order:
      //   0 dz(p0) 1 x(8-t, p0) 2 x(8-t, p1) 3 dz(p1) 4 dz(p2) 5 x(4, v1) 6 dz(p3)
      //   7..10 x(t, p0..p3) 11 x(4, u0)
      // The registers of the stream come from accumulating the transposed products into
      // acc[a][b] with the x(8-t) operand negated (bf16 sign flips, exact) instead of into
      // separate Y^T tiles: 40 accumulator VGPRs instead of 72 (acc[4..7] unused).  No row guard: rows past `rows` (the
      // image's last band when H % 4 != 0) are outside the image, where the dz tile is
      // zero (zero-page DMA, zero mask words), so their products add zeros.
      auto mfma_band_pair = [&](auto bo) {
        constexpr int BO = decltype(bo)::value, NF = 12, P = 3;
        bf16x8 F[BR * NF];  // compile-time indices only: registers, allocated by liveness
        auto rd = [&](auto jc) {
          constexpr int j = decltype(jc)::value, k = j % NF, R = BO + (j / NF) * LL::ROWB;
          if constexpr (k == 0 || k == 3 || k == 4 || k == 6)
            F[j] = tr_pair_px<R>(offB[0] ^ pr.sh(k == 0 ? 0 : k == 3 ? 1 : k == 4 ? 2 : 3));
          else if constexpr (k == 1 || k == 2) F[j] = tr_pair_px<R>(offA[k]);
          else if constexpr (k == 5) F[j] = tr_pair_px<R>(offA[4]);
          else if constexpr (k < 11) F[j] = tr_pair_px<R>(offA[0] ^ pr.sh(k - 7));
          else F[j] = tr_pair_px<R>(offA[3]);
        };
        // group g of a row first needs fragment pf_last(g); reads up to that + P are issued before it
        static_for<0, BR>([&](auto rc) {
          constexpr int r = decltype(rc)::value, b = r * NF;
          bf16x8 nxa, nxb;
          static_for<0, 9>([&](auto gc) {
            constexpr int g = decltype(gc)::value;
            constexpr int lo = g == 0 ? (r == 0 ? 0 : cmin(BR * NF, b - NF + pf_last(8) + 1 + P))
                                      : cmin(BR * NF, b + pf_last(g - 1) + 1 + P);
            constexpr int hi = cmin(BR * NF, b + pf_last(g) + 1 + P);
            static_for<lo, hi>(rd);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (g == 0) {
              nxa = neg_bf16x8(F[b + 1]);
              nxb = neg_bf16x8(F[b + 2]);
            }
            if constexpr (g < 4) {  // transposed products of tap 8-t (+ the tap-4 partner's)
              constexpr int dzk = g == 0 ? 0 : g == 1 ? 3 : g == 2 ? 4 : 6;
              acc[g][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(F[b + dzk], nxa, acc[g][0], 0, 0, 0);
              acc[g][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(F[b + dzk], nxb, acc[g][1], 0, 0, 0);
              if constexpr (g == 2) {  // dz(perm[s1]) x x(4, v1)
                const bf16x8 sel = pr.s1_is_2() ? F[b + 4] : F[b + 3];
                acc[8][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sel, F[b + 5], acc[8][1], 0, 0, 0);
              }
            } else if constexpr (g < 8) {  // direct products of tap t
              acc[g - 4][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(F[b + 3 + g], F[b], acc[g - 4][0], 0, 0, 0);
              acc[g - 4][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(F[b + 3 + g], F[b + 3], acc[g - 4][1], 0, 0, 0);
            } else {  // the tap-4 tile, db
              acc[8][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(F[b + 11], F[b], acc[8][0], 0, 0, 0);
              if (dbw) {
                accb[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, F[b], accb[0], 0, 0, 0);
                accb[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, F[b + 3], accb[1], 0, 0, 0);
              }
            }
          });
        });
      };
      auto convert_next = [&]() {  // the next band's dz of this wave's own row
        if (more) {
          vm_wait(0);  // own dy row and mask dwords of band it+1 (x DMA and fold loads too)
          if (wave == 4) ASR_BTR(1, 1, it, 4);
          convert_own(orow, buf ^ 1, mwv);
        }
      };
      auto mfma_band = [&](auto bo) {
        if constexpr (PAIR) mfma_band_pair(bo);
        else mfma_band_full(bo);
      };
      if (it > 0) {
        const unsigned dlt = buf ? (unsigned)LL::TILE : (unsigned)-LL::TILE;
#pragma unroll
        for (int k = 0; k < NOA; ++k) offA[k] += dlt;
#pragma unroll
        for (int k = 0; k < NOB; ++k) offB[k] += dlt;
      }
      mfma_band(std::integral_constant<int, 0>{});
      if (wave == 4) ASR_BTR(1, 1, it, 3);
      convert_next();
      if (wave == 4) ASR_BTR(1, 1, it, 5);
      if (RK2 && cont) {  // halo rows of the next band of this image (Euler: the dgrad waves copy them)
        // compiler-visible LDS accesses: the item's DMAs were retired by the vm_wait(0)
        // before the convert (cont implies more), so hipcc's own waits cost nothing
        // here, and a copied or spilled read result stays correct
        const unsigned base = lds_u32(lds);
        const int nbf = buf ^ 1;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int c = ft + 512 * k;
          if (c < 5 * 256) {
            const int which = c >> 8;
            const unsigned o = (unsigned)((c & 255) + NQ) * 16u;
            const unsigned sreg = which < 2 ? LL::DZ : which < 4 ? LL::X : LL::DY;
            const int srow = which == 4 ? BR + 1 : BR + (which & 1);
            const int drow = which == 4 ? 1 : (which & 1);
            lds_st128(base + sreg + nbf * LL::TILE + drow * LL::ROWB + o,
                      lds_ld128(base + sreg + buf * LL::TILE + srow * LL::ROWB + o));
          }
        }
      }
#pragma unroll
      for (int q = 0; q < 2; ++q)
        if (fold && fp < fpe) {
          facc += fv[q];
          ++fp;
          foff += ES;
        }
      const bool last_of_stage = cur.b == nb - 1 && cur.n == n1 - 1;
      const bool last_of_block = last_of_stage && !(RK2 && (cur.l & 1));
      if (RK2 && last_of_stage && (cur.l & 1)) {  // second -> first RK2 stage of the block: acc *= 2 (exact)
#pragma unroll
        for (int mi = 0; mi < MTW; ++mi) acc[mi][0] *= 2.f, acc[mi][1] *= 2.f;
        accb[0] *= 2.f, accb[1] *= 2.f;
      }
      if (last_of_block) {
        if (l + 2 < L && l + 2 >= lfold) fold_end(l + 2);
        // publish block l's dW tiles and db (write-through; drained at the next band barrier)
        float* slab = slabs + (long)l * slab_stride + (long)blockIdx.x * ES;
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(slab, 0, ES * 4, 0x00020000);
        auto put = [&](int tile, f32x4 v) {
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, ((tile * 64 + lane) * 4) * 4, 0, 16);
        };
        if constexpr (PAIR) {  // D = X - Y^T per pair tile: 8 (+1 or 2 tap-4) tiles of the 74
#pragma unroll
          for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
              put(pr.tile(a, b), acc[a][b] * hsb);
          if (pr.self()) {
            put(PairSlab::kSelf + pr.perm(0), acc[8][0] * hsb);  // raw X(4, c, c), c even
            put(PairSlab::kSelf + pr.perm(1), acc[8][1] * hsb);  // X(4, c, c)^T, c odd
          } else {
            put(PairSlab::kTap4 + pr.k4(), (acc[8][0] - acc[8][1]) * hsb);
          }
#pragma unroll
          for (int mi = 0; mi < MTW; ++mi) acc[mi][0] = acc[mi][1] = f32x4{0.f, 0.f, 0.f, 0.f};
        } else {
#pragma unroll
          for (int mi = 0; mi < MTW; ++mi)
#pragma unroll
            for (int oi = 0; oi < 2; ++oi) {
              const int mt = tg * MTW + mi;
              put(mt * 4 + oq + oi, acc[mi][oi] * hsb);
              acc[mi][oi] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
        if (dbw) {
          if (g == 0) {
#pragma unroll
            for (int oi = 0; oi < 2; ++oi) {
              const int ob = PAIR ? pr.perm(oi) : oq + oi;
              __hip_atomic_store((gf32*)(slab + (ES - C) + 16 * ob + lx), hsb * accb[oi][0], __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
            }
          }
          accb[0] = accb[1] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
      if (wave == 4) ASR_BTR(1, 1, it, 6);
      cur = nxt;
      adv(nxt);
    }
    barrier_vm(0);
  }
  ASR_BCLK(1, 1);
}

// ===========================================================================
// Stem weight gradient on MFMA (C = 16 or 64, CIN=3, W=32, H % 8 == 0), from dz1 =
// dx1 * [x1 > 0] (written by the first block's backward, k_bwd3<..., RO> or k_bwd3_stack with ro0):
//   dW1[kappa][o] = inv_std * sum_p (img[p + tap] - mean)[ci] * dz1[p][o]
//   db1[o]        = sum_p dz1[p][o]
// (models/tfkeras_resnets.py:555-572: input normalisation, then the 3x3 SAME
// conv1 + relu).  K = pixels (one image row per k-step), M = kappa = tap*3 +
// ci (27, a row of ones at 27 for db1, padded to 32), N = o.  The image's
// im2col sits in LDS as a 32-channel tile of bf16 (v - mean): exact for u8
// input with a half-integer mean, so the bf16 products are exact and only
// the fp32 accumulation rounds.  dz1 rows stream in by LDS-DMA, 8-row bands
// double-buffered; both operands come from transposed LDS reads exactly as
// in the blocks' weight gradient.  One slab [dW1 (27*C) | db1 (C)] per WG.
// ===========================================================================
template <int C, typename Tin>
__global__ __launch_bounds__(256) void k_stem_wgrad_mfma(const Tin* __restrict__ img, const bf16* __restrict__ dz1,
                                                         int N, int H, float mean, float inv_std,
                                                         float* __restrict__ slabs) {
  constexpr int W = 32, CIN = 3, TW = W + 2, BRS = 8, KC = 9 * CIN, NT = C / 16;
  constexpr int IMROW = TW * 4 * 16, DZROW = TW * (C / 8) * 16, DZT = BRS * DZROW;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int IM = 0, DZ0 = H * IMROW, FT = DZ0 + 2 * DZT;  // im2col | 2 dz1 bands | staged image (fp32, halo)
  float* ft = (float*)(lds + FT);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, lx = lane & 15, tq = lx >> 2, tp = lx & 3;
  const int nbands = H / BRS;
  for (int i = tid; i < (H + 2) * TW * CIN; i += 256) ft[i] = 0.f;  // halo stays zero
  f32x4 acc[2][NT];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int n0 = blockIdx.x, items = ((N - n0 + (int)gridDim.x - 1) / (int)gridDim.x) * nbands;
  auto band_n = [&](int it) { return n0 + (it / nbands) * (int)gridDim.x; };
  auto dma_band = [&](int it, int buf) {
    dma_rows<C, W>(dz1, lds + DZ0 + buf * DZT, band_n(it), (it % nbands) * BRS, BRS, H, wave, 4, lane);
  };
  if (items > 0) dma_band(0, 0);
  for (int it = 0; it < items; ++it) {
    const int buf = it & 1, b = it % nbands;
    if (b == 0) {  // a new image: stage it (fp32, v - mean) and build its im2col
      const int n = band_n(it);
      __syncthreads();  // the previous image's im2col fully read
      const Tin* src = img + (long)n * H * W * CIN;
      for (int i = tid; i < H * W * CIN; i += 256) {
        const int ci = i % CIN, p = i / CIN;
        ft[((p / W + 1) * TW + p % W + 1) * CIN + ci] = (float)src[i] - mean;
      }
      __syncthreads();
      for (int p = tid; p < H * W; p += 256) {
        const int y = p / W, x = p % W;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          bf16x8 v;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int kap = 8 * q + j;
            float f = 0.f;
            if (kap < KC) {
              const int tap = kap / CIN, ci = kap % CIN;
              f = ft[((y + tap / 3) * TW + x + tap % 3) * CIN + ci];
            } else if (kap == KC) {
              f = 1.f;  // db1 row
            }
            v[j] = (bf16)f;
          }
          *(bf16x8*)(lds + IM + toff<32>(y, x + 1, q, TW)) = v;
        }
      }
    }
    barrier_vm(0);  // band it landed (and the im2col is written)
    if (it + 1 < items) dma_band(it + 1, buf ^ 1);
    const unsigned char* dzt = lds + DZ0 + buf * DZT;
#pragma unroll
    for (int k = 0; k < BRS / 4; ++k) {  // this wave's rows of the band
      const int r = wave + 4 * k, y = b * BRS + r;
      const int pb = 8 * g + tq;
      bf16x8 A[2], B[NT];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int q = 2 * mt + (tp >> 1);
        A[mt] = tr_pair(lds + IM + toff<32>(y, pb + 1, q, TW) + 8 * (tp & 1),
                        lds + IM + toff<32>(y, pb + 5, q, TW) + 8 * (tp & 1));
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int q = 2 * nt + (tp >> 1);
        B[nt] = tr_pair(dzt + toff<C>(r, pb + 1, q, TW) + 8 * (tp & 1), dzt + toff<C>(r, pb + 5, q, TW) + 8 * (tp & 1));
      }
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[mt], B[nt], acc[mt][nt], 0, 0, 0);
    }
  }
  // the 4 waves' partials, summed in a fixed order (deterministic)
  barrier_vm(0);
  float* red = (float*)lds;  // [4 waves][32 m][C]
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int e = 0; e < 4; ++e) red[(wave * 32 + 16 * mt + 4 * g + e) * C + 16 * nt + lx] = acc[mt][nt][e];
  __syncthreads();
  float* slab = slabs + (long)blockIdx.x * (KC * C + C);
  for (int i = tid; i < (KC + 1) * C; i += 256) {
    const float v = (red[i] + red[32 * C + i]) + (red[2 * 32 * C + i] + red[3 * 32 * C + i]);
    slab[i] = i < KC * C ? v * inv_std : v;  // rows 0..26 dW1, row 27 db1
  }
}

// ===========================================================================
// Stem forward on MFMA (C = 16 or 64, CIN=3, W=32): x1 = relu(conv3x3((v - mean) *
// inv_std, W1) + b1), bf16 NHWC out (models/tfkeras_resnets.py:555-572).
// M = o (C/16 tiles), K = kappa = tap*3 + ci (27, padded to 32: one k-step),
// N = 16 pixels.  B: lane (pixel lx, kappa 8g..8g+7) gathers its 8 patch
// values from the image staged in LDS as fp32 v - mean (bf16-exact for u8
// input with a half-integer mean); A = inv_std * W1^T split into bf16 hi +
// lo parts held in registers (two MFMAs per tile: W1 to ~16 mantissa bits,
// so the result matches the fp32 VALU kernel to accumulation-order noise).
// Epilogue: + b1 (fp32), relu, bf16, 16-B stores at C=64 (a 16-lane row swap
// between o-tile pairs gives each lane 8 consecutive channels), 8-B stores at
// C=16 (one o-tile: 16 pixels x 32 B contiguous per tile).
// ===========================================================================
template <int C, typename Tin>
__global__ __launch_bounds__(256) void k_stem_fwd_mfma(const Tin* __restrict__ img, const float* __restrict__ w1,
                                                       const float* __restrict__ b1, int N, int H, float mean,
                                                       float inv_std, bf16* __restrict__ out) {
  constexpr int W = 32, CIN = 3, TW = W + 2, KC = 9 * CIN, MT = C / 16;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  float* ft = (float*)lds;  // staged image (fp32 v - mean), zero halo
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, lx = lane & 15;
  for (int i = tid; i < (H + 2) * TW * CIN; i += 256) ft[i] = 0.f;  // halo stays zero
  // A fragments: lane (o = 16 mt + lx, kappa 8g..8g+7), hi and lo bf16 parts
  bf16x8 Ah[MT], Al[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kap = 8 * g + j;
      const float wv = kap < KC ? w1[kap * C + 16 * mt + lx] * inv_std : 0.f;
      const bf16 hi = (bf16)wv;
      Ah[mt][j] = hi;
      Al[mt][j] = (bf16)(wv - (float)hi);
    }
  float bz[MT][4];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int e = 0; e < 4; ++e) bz[mt][e] = b1 ? b1[16 * mt + 4 * g + e] : 0.f;
  // B operand: lane (pixel lx, kappa 8g..8g+7) read straight from the staged
  // image: tap (ky, kx), channel ci of kappa = offset (ky*TW + kx)*CIN + ci
  int koff[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int kap = min(8 * g + j, KC - 1), tap = kap / CIN, ci = kap % CIN;
    koff[j] = ((tap / 3) * TW + tap % 3) * CIN + ci;
  }
  for (int n = blockIdx.x; n < N; n += gridDim.x) {
    __syncthreads();  // the previous image fully read
    const Tin* src = img + (long)n * H * W * CIN;
    for (int i = tid; i < H * W * CIN; i += 256) {
      const int ci = i % CIN, p = i / CIN;
      ft[((p / W + 1) * TW + p % W + 1) * CIN + ci] = (float)src[i] - mean;
    }
    __syncthreads();
    // pixel tiles: wave w takes tiles w, w+4, ... (16 pixels of one row each)
    for (int pt = wave; pt < H * W / 16; pt += 4) {
      const int y = pt / (W / 16), x0 = (pt % (W / 16)) * 16;
      const float* pb = ft + (y * TW + x0 + lx) * CIN;
      bf16x8 B;
#pragma unroll
      for (int j = 0; j < 8; ++j) B[j] = (bf16)((8 * g + j < KC) ? pb[koff[j]] : 0.f);
      f32x4 acc[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        acc[mt] = f32x4{bz[mt][0], bz[mt][1], bz[mt][2], bz[mt][3]};
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ah[mt], B, acc[mt], 0, 0, 0);
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Al[mt], B, acc[mt], 0, 0, 0);
      }
      // lane (g, lx): channels 16 mt + 4g + e of pixel x0 + lx
      u32x2 ov[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        bf16x4 o4;
#pragma unroll
        for (int e = 0; e < 4; ++e) o4[e] = (bf16)fmaxf(acc[mt][e], 0.f);
        ov[mt] = *(const u32x2*)&o4;
      }
      bf16* orow = out + (((long)n * H + y) * W + x0 + lx) * C;
      if constexpr (MT == 1) {
        *(u32x2*)(orow + 4 * g) = ov[0];
      } else {
#pragma unroll
        for (int mp = 0; mp < MT / 2; ++mp) {  // o-tiles 2mp, 2mp+1 -> lane row g: channels 16(2mp + (g&1)) + 8(g>>1)
          const auto s0 = __builtin_amdgcn_permlane16_swap(ov[2 * mp][0], ov[2 * mp + 1][0], false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(ov[2 * mp][1], ov[2 * mp + 1][1], false, false);
          *(u32x4*)(orow + 16 * (2 * mp + (g & 1)) + 8 * (g >> 1)) = u32x4{s0[0], s1[0], s0[1], s1[1]};
        }
      }
    }
  }
}

}  // namespace blk

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
constexpr int kBwdBR = 4;
constexpr int kFwdBR = 4;  // k_fwd3 / k_fwd3_stack row band
constexpr int kMaxBlockSlabs = 512;

#if ASR_BLK_TRACE
}  // namespace asr
extern "C" int asr_debug_blk_trace(void* trace, size_t tbytes, void* clock, size_t cbytes) {
  if (hipMemcpyFromSymbol(trace, HIP_SYMBOL(asr::blk::g_btrace), tbytes) != hipSuccess) return -1;
  return hipMemcpyFromSymbol(clock, HIP_SYMBOL(asr::blk::g_bclock), cbytes) == hipSuccess ? 0 : -1;
}
extern "C" int asr_debug_blk_switch(void* dst, size_t bytes) {  // g_bswitch (k_bwd3_stack block switches)
  if (bytes > sizeof(asr::blk::g_bswitch)) bytes = sizeof(asr::blk::g_bswitch);
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(asr::blk::g_bswitch), bytes) == hipSuccess ? 0 : -1;
}
namespace asr {
#endif

static int persistent_grid(long items) {
  int cus = cu_count();
  if (cus <= 0) cus = 256;
  return (int)std::max<long>(1, std::min<long>({items, (long)cus, (long)kMaxBlockSlabs}));
}

template <int C, int W, int BR, int NW>
static int launch_fwd_v(int mode, const void* x, const void* resid, void* y, uint8_t* mask, const void* w,
                        const float* bias, float h, int N, int H, hipStream_t s) {
  static_assert(NW % blk::Geo<C>::OSPLIT == 0, "waves must cover the o-split");
  const long items = (long)N * ((H + BR - 1) / BR);
  if (items > 0x7fffffffL) return fail(ASR_E_UNSUPPORTED, "bf16 block: too many row bands (%ld)", items);
  int cus = cu_count();
  if (cus <= 0) cus = 256;
  const int grid = (int)std::max<long>(1, std::min<long>(items, (long)cus * (8 / NW)));
  const size_t lds = 2 * (size_t)(BR + 2) * (W + 2) * C * 2;
  if constexpr (C == 64 && W == 32 && BR == 4 && NW == 4) {
    if (!resid || mode == blk::FWD_EULER) {
      const int grid3 = (int)std::max<long>(1, std::min<long>(items, (long)cus * kFwd3Wgs));
      if (mode == blk::FWD_EULER && resid)
        hipLaunchKernelGGL((blk::k_fwd3<C, W, BR, blk::FWD_EULER, 3, true>), dim3(grid3), dim3(256), lds, s,
                           (const bf16*)x, (const bf16*)resid, (bf16*)y, mask, (const bf16*)w, bias, h, N, H);
      else if (mode == blk::FWD_EULER)
        hipLaunchKernelGGL((blk::k_fwd3<C, W, BR, blk::FWD_EULER, 3>), dim3(grid3), dim3(256), lds, s, (const bf16*)x,
                           nullptr, (bf16*)y, mask, (const bf16*)w, bias, h, N, H);
      else
        hipLaunchKernelGGL((blk::k_fwd3<C, W, BR, blk::FWD_CONV, 3>), dim3(grid3), dim3(256), lds, s, (const bf16*)x,
                           nullptr, (bf16*)y, mask, (const bf16*)w, bias, h, N, H);
      ASR_LAUNCH_CHECK("k_fwd3");
      return ASR_OK;
    }
  }
  if constexpr (C >= 32) {
    if (mode == blk::FWD_EULER && resid) {  // second RK2 stage: residual from the step input
      hipLaunchKernelGGL((blk::k_fwd_pipe<C, W, BR, blk::FWD_EULER, NW, true>), dim3(grid), dim3(64 * NW), lds, s,
                         (const bf16*)x, (const bf16*)resid, (bf16*)y, mask, (const bf16*)w, bias, h, N, H);
    } else if (mode == blk::FWD_EULER) {
      hipLaunchKernelGGL((blk::k_fwd_pipe<C, W, BR, blk::FWD_EULER, NW>), dim3(grid), dim3(64 * NW), lds, s,
                         (const bf16*)x, nullptr, (bf16*)y, mask, (const bf16*)w, bias, h, N, H);
    } else {
      hipLaunchKernelGGL((blk::k_fwd_pipe<C, W, BR, blk::FWD_CONV, NW>), dim3(grid), dim3(64 * NW), lds, s,
                         (const bf16*)x, nullptr, (bf16*)y, mask, (const bf16*)w, bias, h, N, H);
    }
  } else {
    if (mode == blk::FWD_EULER)
      hipLaunchKernelGGL((blk::k_fwd<C, W, BR, blk::FWD_EULER, NW>), dim3(grid), dim3(64 * NW), lds, s,
                         (const bf16*)x, (const bf16*)resid, (bf16*)y, mask, (const bf16*)w, bias, h, N, H);
    else
      hipLaunchKernelGGL((blk::k_fwd<C, W, BR, blk::FWD_CONV, NW>), dim3(grid), dim3(64 * NW), lds, s,
                         (const bf16*)x, (const bf16*)resid, (bf16*)y, mask, (const bf16*)w, bias, h, N, H);
  }
  ASR_LAUNCH_CHECK("k_fwd");
  return ASR_OK;
}

template <int C, int W>
static int launch_fwd(int mode, const void* x, const void* resid, void* y, uint8_t* mask, const void* w,
                      const float* bias, float h, int N, int H, hipStream_t s) {
  // 4-row bands, 4 waves (one 16-channel o-tile each at C=64), 2 WGs per CU
  // (geometry chosen by A/B on MI355X against 8x8, 4x8 and 8x4)
  return launch_fwd_v<C, W, 4, 4>(mode, x, resid, y, mask, w, bias, h, N, H, s);
}

template <int C, int W>
static int launch_bwd(int mode, const void* dy, const void* x, const uint8_t* mask, const void* w, float h,
                      float two_gamma, int N, int H, void* dx, float* slabs, int* nslabs, const void* extra,
                      int skip_dy, int relu_dx, int* relu_done, const float* fold_slabs, int fold_P, float* fold_grp,
                      int* fold_done, int accum, hipStream_t s) {
  const long items = (long)N * ((H + kBwdBR - 1) / kBwdBR);
  if (items > 0x7fffffffL) return fail(ASR_E_UNSUPPORTED, "bf16 block: too many row bands (%ld)", items);
  const int grid = persistent_grid(items);
  *nslabs = grid;
  using L = blk::BwdLds<C, W, kBwdBR>;
  const size_t red = (size_t)(12288 + 4 * 64) * 4;
  const size_t lds = std::max((size_t)(extra ? L::TOTAL_XT : L::TOTAL), red);
#define ASR_LAUNCH_BWD(M, XT)                                                                                    \
  hipLaunchKernelGGL((blk::k_bwd<C, W, kBwdBR, M, XT>), dim3(grid), dim3(512), lds, s, (const bf16*)dy, (const bf16*)x, \
                     mask, (const bf16*)w, h, two_gamma, N, H, (bf16*)dx, slabs, (const bf16*)extra, skip_dy, accum)
  const bool xt = extra != nullptr || skip_dy != 0 || accum != 0;
  if constexpr (C == 64) {
    // v2: the Euler block, the plain conv, and both RK2 stages (the first: extra
    // dx term + slab accumulation); other compositions run the v1 kernel
    const bool xt2 = extra && accum && !skip_dy && mode == blk::BWD_EULER && !relu_dx;
    if (xt2 || (!extra && !accum && (mode == blk::BWD_EULER || !skip_dy))) {
      using L2 = blk::Bwd2Lds<C, W, kBwdBR>;
      const size_t lds2 = std::max((size_t)L2::TOTAL, red);
      // the folded pass gives each thread one 16-B chunk: at most 512 per WG
      const long fchunks = (long)((fold_P + 31) / 32) * ((9 * C * C + C) / 4);
      if ((fchunks + grid - 1) / grid > 512) fold_P = 0;
#define ASR_LAUNCH_BWD3(M, RO, XT)                                                                            \
  hipLaunchKernelGGL((blk::k_bwd3<C, W, kBwdBR, M, RO, XT>), dim3(grid), dim3(768), lds2, s, (const bf16*)dy,    \
                     (const bf16*)x, mask, (const bf16*)w, h, two_gamma, N, H, (bf16*)dx, slabs, fold_slabs, fold_P, \
                     fold_grp, skip_dy, (const bf16*)extra)
      if (xt2) ASR_LAUNCH_BWD3(blk::BWD_EULER, false, true);
      else if (mode == blk::BWD_EULER && relu_dx) {
        ASR_LAUNCH_BWD3(blk::BWD_EULER, true, false);
        if (relu_done) *relu_done = 1;
      } else if (mode == blk::BWD_EULER) ASR_LAUNCH_BWD3(blk::BWD_EULER, false, false);
      else ASR_LAUNCH_BWD3(blk::BWD_CONV, false, false);
#undef ASR_LAUNCH_BWD3
      ASR_LAUNCH_CHECK("k_bwd3");
      if (fold_done) *fold_done = fold_P > 0;
      return ASR_OK;
    }
  }
  if (mode == blk::BWD_EULER) {
    if (xt) ASR_LAUNCH_BWD(blk::BWD_EULER, true);
    else ASR_LAUNCH_BWD(blk::BWD_EULER, false);
  } else {
    if (xt) ASR_LAUNCH_BWD(blk::BWD_CONV, true);
    else ASR_LAUNCH_BWD(blk::BWD_CONV, false);
  }
#undef ASR_LAUNCH_BWD
  ASR_LAUNCH_CHECK("k_bwd");
  return ASR_OK;
}

// ---------------------------------------------------------------------------
// stem weight gradient on MFMA (see k_stem_wgrad_mfma)
// ---------------------------------------------------------------------------
static size_t stem_wgrad_mfma_lds(int H, int C) {
  return (size_t)H * 34 * 64 + 2 * 8 * 34 * (C / 8) * 16 + (size_t)(H + 2) * 34 * 3 * 4;
}

bool stem_wgrad_mfma_supported(int Cin, int H, int W, int C) {
  return Cin == 3 && W == 32 && (C == 64 || C == 16) && H % 8 == 0 && H >= 8 &&
         stem_wgrad_mfma_lds(H, C) <= 160 * 1024;
}

int stem_wgrad_mfma(const void* img, int input_u8, const void* dz1, int N, int H, int W, int Cin, int C, float mean,
                    float inv_std, int use_norm, float* slabs, int* nslabs, hipStream_t s) {
  if (!stem_wgrad_mfma_supported(Cin, H, W, C)) return fail(ASR_E_UNSUPPORTED, "stem wgrad (MFMA): unsupported shape");
  int cus = cu_count();
  if (cus <= 0) cus = 256;
  const int grid = std::max(1, std::min(N, std::min(cus, kMaxBlockSlabs)));
  *nslabs = grid;
  const size_t lds = std::max(stem_wgrad_mfma_lds(H, C), (size_t)4 * 32 * C * 4);  // (reduction area)
  const float m = use_norm ? mean : 0.f, is = use_norm ? inv_std : 1.f;
#define ASR_STEMW(CC, TI)                                                                                   \
  hipLaunchKernelGGL((blk::k_stem_wgrad_mfma<CC, TI>), dim3(grid), dim3(256), lds, s, (const TI*)img, \
                     (const bf16*)dz1, N, H, m, is, slabs)
  if (C == 64) {
    if (input_u8) ASR_STEMW(64, uint8_t);
    else ASR_STEMW(64, float);
  } else {
    if (input_u8) ASR_STEMW(16, uint8_t);
    else ASR_STEMW(16, float);
  }
#undef ASR_STEMW
  ASR_LAUNCH_CHECK("k_stem_wgrad_mfma");
  return ASR_OK;
}

bool stem_fwd_mfma_supported(int Cin, int H, int W, int C) {
  const size_t lds = (size_t)(H + 2) * 34 * 3 * 4;
  return Cin == 3 && W == 32 && (C == 64 || C == 16) && H >= 1 && lds <= 160 * 1024;
}

int stem_fwd_mfma(const void* img, int input_u8, const float* w1, const float* b1, int N, int H, int W, int Cin, int C,
                  float mean, float inv_std, int use_norm, void* out, hipStream_t s) {
  if (!stem_fwd_mfma_supported(Cin, H, W, C)) return fail(ASR_E_UNSUPPORTED, "stem fwd (MFMA): unsupported shape");
  int cus = cu_count();
  if (cus <= 0) cus = 256;
  const int grid = std::max(1, std::min(N, 4 * cus));
  const size_t lds = (size_t)(H + 2) * 34 * 3 * 4;
  const float m = use_norm ? mean : 0.f, is = use_norm ? inv_std : 1.f;
#define ASR_STEMF(CC, TI)                                                                                     \
  hipLaunchKernelGGL((blk::k_stem_fwd_mfma<CC, TI>), dim3(grid), dim3(256), lds, s, (const TI*)img, w1, b1, N, H, m, \
                     is, (bf16*)out)
  if (C == 64) {
    if (input_u8) ASR_STEMF(64, uint8_t);
    else ASR_STEMF(64, float);
  } else {
    if (input_u8) ASR_STEMF(16, uint8_t);
    else ASR_STEMF(16, float);
  }
#undef ASR_STEMF
  ASR_LAUNCH_CHECK("k_stem_fwd_mfma");
  return ASR_OK;
}

int block_fwd_mfma(int mode, const void* x, const void* resid, void* y, uint8_t* mask, const void* w,
                   const float* bias, float h, int N, int H, int W, int C, hipStream_t s) {
  if (W != 32) return fail(ASR_E_UNSUPPORTED, "bf16 block: W=%d not supported (W must be 32)", W);
  switch (C) {
    case 16: return launch_fwd<16, 32>(mode, x, resid, y, mask, w, bias, h, N, H, s);
    case 32: return launch_fwd<32, 32>(mode, x, resid, y, mask, w, bias, h, N, H, s);
    case 64: return launch_fwd<64, 32>(mode, x, resid, y, mask, w, bias, h, N, H, s);
  }
  return fail(ASR_E_UNSUPPORTED, "bf16 block: C=%d not supported (16, 32, 64)", C);
}

// RK2: 2L stages in one launch (k_fwd3_stack<..., RK2>): x_l -> xmid_l (xm + l*y_stride,
// mask1 at masks + l*mask_stride) -> x_{l+1} (mask2 at masks2 + l*mask_stride)
int block_stack_fwd_rk2_mfma(const void* x0, void* ys, void* xm, long y_stride, uint8_t* masks, uint8_t* masks2,
                             long mask_stride, const void* w, long w_stride, const float* bias, long bias_stride,
                             float h, int N, int H, int W, int C, int L, hipStream_t s);

bool block_stack_fwd_supported(int N, int H, int W, int C) {
  return C == 64 && W == 32 && N >= 1 && (H + kFwdBR - 1) / kFwdBR >= 4;
}

// all L Euler blocks in one launch (k_fwd3_stack); x_l of block l >= 1 is
// ys + (l-1)*y_stride, its output ys + l*y_stride (elements)
int block_stack_fwd_mfma(const void* x0, void* ys, long y_stride, uint8_t* masks, long mask_stride, const void* w,
                         long w_stride, const float* bias, long bias_stride, float h, int N, int H, int W, int C, int L,
                         hipStream_t s, int slots) {
  if (!block_stack_fwd_supported(N, H, W, C) || L < 1)
    return fail(ASR_E_UNSUPPORTED, "stack forward: needs C=64, W=32, >= 4 row bands per image (C=%d W=%d H=%d)", C, W, H);
  if (y_stride < (long)N * H * W * C) return fail(ASR_E_ARG, "stack forward: y_stride smaller than one activation");
  if (slots != 0 && slots != 2) return fail(ASR_E_ARG, "stack forward: slots must be 0 or 2");
  int cus = cu_count();
  if (cus <= 0) cus = 256;
  const int grid = std::max(1, std::min(N, 2 * cus));
  const size_t lds = 3 * (size_t)(kFwdBR + 2) * (W + 2) * C * 2;  // k_fwd3_stack's ring of three tiles
  hipLaunchKernelGGL((blk::k_fwd3_stack<64, 32, kFwdBR>), dim3(grid), dim3(256), lds, s, (const bf16*)x0,
                     (bf16*)ys, y_stride, masks, mask_stride, (const bf16*)w, w_stride, bias, bias_stride, h, N, H, L,
                     slots);
  ASR_LAUNCH_CHECK("k_fwd3_stack");
  return ASR_OK;
}

// test knobs (asr_debug_stack_backward): a forced grid (0: one workgroup per
// CU) and the bound of the slab hand-off's wait (0: the default)
static int g_stack_grid_override = 0;

// dynamic LDS of k_bwd3_stack: the v2 tiles + mask table, then its "late" word
static size_t stack_bwd_lds() { return (size_t)blk::Bwd2Lds<64, 32, kBwdBR>::TOTAL + 16; }

// k_bwd3_stack workgroups the device keeps resident per CU (both
// instantiations; cached per device): the in-launch hand-off is fast only with
// the whole grid resident, so the stacked path is used only when this is >= 1
static int stack_bwd_resident_per_cu() {
  static int dev_cached = -1, per = 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (dev != dev_cached) {
    int a = 0, b = 0, c = 0, d = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, blk::k_bwd3_stack<64, 32, kBwdBR, false, false>, 768,
                                                     stack_bwd_lds()) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, blk::k_bwd3_stack<64, 32, kBwdBR, true, false>, 768,
                                                     stack_bwd_lds()) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&c, blk::k_bwd3_stack<64, 32, kBwdBR, false, true>, 768,
                                                     stack_bwd_lds()) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&d, blk::k_bwd3_stack<64, 32, kBwdBR, true, true>, 768,
                                                     stack_bwd_lds()) != hipSuccess)
      return 0;
    per = std::min(std::min(a, b), std::min(c, d));
    dev_cached = dev;
  }
  return per;
}

bool block_stack_bwd_supported(int N, int H, int W, int C) {
  return C == 64 && W == 32 && N >= 1 && (H + kBwdBR - 1) / kBwdBR >= 4 && stack_bwd_resident_per_cu() >= 1;
}

// workgroups of k_bwd3_stack: one per CU at most (the in-launch slab
// hand-off needs every workgroup resident), whole images each
int block_stack_bwd_grid(int N) {
  int cus = cu_count();
  if (cus <= 0) cus = 256;
  const int cap = g_stack_grid_override > 0 ? g_stack_grid_override : cus;
  return std::max(1, std::min(N, std::min(cap, kMaxBlockSlabs)));
}

int stack_done_words(int L) { return 2 * L + 4; }

// floats per slab of k_bwd3_stack: the full dW (9C^2 + C) or, pair-local, the 74 D tiles + db
long stack_slab_floats(int C, int pair) { return pair ? (long)PairSlabLayout::ES : 9L * C * C + C; }

// the backward of L Euler blocks in one launch (k_bwd3_stack).  dbuf0 holds
// dL/dx_L on entry, or gtop (Euler) its per-image row (the head's GAP
// gradient, bf16 [N][C]): then dbuf0 is not read.  Block 0's dx ends in dbuf[L & 1].  Block l's slabs (grid
// of them, tile-major dW) at slabs + l*slab_stride; blocks >= lfold leave as
// 32-slab group sums at grp + l*grp_stride (unless flagged), the rest as slabs:
// stack_bwd_reduce_rest finishes both.  done: stack_done_words(L) words, zeroed
// here: the per-block publish counters [0, L+4) and the per-block flags
// [L+4, 2L+4) of folds whose wait ran out.
int block_stack_bwd_mfma(void* dbuf0, void* dbuf1, const void* xs, long x_stride, const uint8_t* masks,
                         long mask_stride, const void* w, long w_stride, float h, float two_gamma, int N, int H, int W,
                         int C, int L, int ro0, float* slabs, long slab_stride, float* grp, long grp_stride,
                         unsigned* done, int* lfold_out, hipStream_t s, const void* xm, const uint8_t* masks2,
                         void* gbuf, const void* gtop, int fold, int pair) {
  if (!block_stack_bwd_supported(N, H, W, C) || L < 1)
    return fail(ASR_E_UNSUPPORTED, "stack backward: needs C=64, W=32, >= 4 row bands per image (C=%d W=%d H=%d)", C, W, H);
  const int grid = block_stack_bwd_grid(N);
  const long ES = stack_slab_floats(C, pair);
  if (slab_stride < (long)grid * ES) return fail(ASR_E_ARG, "stack backward: slab_stride too small");
  // in-kernel pass 1 needs <= 512 group-row chunks per workgroup (one per wgrad thread)
  const long fchunks = (long)((grid + 31) / 32) * (ES / 4);
  // fold = 0: no in-launch pass 1, so no workgroup ever waits for another (no
  // co-residency needed: e.g. several processes sharing one device)
  const int lfold = fold && (fchunks + grid - 1) / grid <= 512 ? 2 : L;
  if (lfold_out) *lfold_out = lfold;
  ASR_TRY(hip_check(hipMemsetAsync(done, 0, (size_t)stack_done_words(L) * 4, s), "hipMemsetAsync"));
  unsigned* skipf = done + L + 4;
  const size_t lds = stack_bwd_lds();
#define ASR_STACK_BWD(RK, PR)                                                                                   \
  hipLaunchKernelGGL((blk::k_bwd3_stack<64, 32, kBwdBR, RK, PR>), dim3(grid), dim3(768), lds, s, (bf16*)dbuf0,         \
                     (bf16*)dbuf1, (const bf16*)xs, x_stride, masks, mask_stride, (const bf16*)w, w_stride, h,         \
                     two_gamma, N, H, L, RK ? 0 : ro0, slabs, slab_stride, grp, grp_stride, done, skipf, lfold,        \
                     RK ? (const bf16*)xm : nullptr, RK ? masks2 : nullptr, RK ? (bf16*)gbuf : nullptr,                \
                     RK ? nullptr : (const bf16*)gtop)
  if (xm) {  // RK2: both stages of every block (x_mid stack at xm, stride x_stride; masks2; g scratch)
    if (!masks2 || !gbuf) return fail(ASR_E_ARG, "stack backward (RK2): masks2 and the g buffer are required");
    if (pair) ASR_STACK_BWD(true, true);
    else ASR_STACK_BWD(true, false);
  } else {
    if (pair) ASR_STACK_BWD(false, true);
    else ASR_STACK_BWD(false, false);
  }
#undef ASR_STACK_BWD
  ASR_LAUNCH_CHECK("k_bwd3_stack");
  return ASR_OK;
}

// Pass 1 of the stacked backward's weight-gradient reduction left after the
// launch: blocks below lfold always, blocks at or above it only where a fold's
// wait ran out (flags[l] != 0: their group rows are recomputed from the slabs,
// all published by now).  Same sums in the same order as k_reduce_slabs and
// the in-launch fold (32-slab groups): deterministic either way.
__global__ __launch_bounds__(256) void k_reduce_slabs_flagged(const float* __restrict__ slabs, long slab_stride, long ES,
                                                              int P, float* __restrict__ grp, long grp_stride, int L,
                                                              int lfold, const unsigned* __restrict__ flags) {
  const long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const int g = blockIdx.y;
  const int p0 = 32 * g, p1 = min(P, p0 + 32);
  for (int l = 0; l < L; ++l) {
    if (l >= lfold && flags[l] == 0u) continue;
    if (e >= ES) continue;
    const float* in = slabs + (long)l * slab_stride;
    float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
    int p = p0;
    for (; p + 3 < p1; p += 4) {
      acc0 += in[(long)p * ES + e];
      acc1 += in[(long)(p + 1) * ES + e];
      acc2 += in[(long)(p + 2) * ES + e];
      acc3 += in[(long)(p + 3) * ES + e];
    }
    for (; p < p1; ++p) acc0 += in[(long)p * ES + e];
    grp[(long)l * grp_stride + (long)g * ES + e] = (acc0 + acc1) + (acc2 + acc3);
  }
}

int stack_bwd_reduce_rest(const float* slabs, long slab_stride, int grid, long ES, float* grp, long grp_stride, int L,
                          int lfold, const unsigned* done, hipStream_t s) {
  const int G = (grid + 31) / 32;
  hipLaunchKernelGGL(k_reduce_slabs_flagged, dim3((unsigned)((ES + 255) / 256), G), dim3(256), 0, s, slabs,
                     slab_stride, ES, grid, grp, grp_stride, L, lfold, done + L + 4);
  ASR_LAUNCH_CHECK("k_reduce_slabs_flagged");
  return ASR_OK;
}

int block_stack_fwd_rk2_mfma(const void* x0, void* ys, void* xm, long y_stride, uint8_t* masks, uint8_t* masks2,
                             long mask_stride, const void* w, long w_stride, const float* bias, long bias_stride,
                             float h, int N, int H, int W, int C, int L, hipStream_t s) {
  if (!block_stack_fwd_supported(N, H, W, C) || L < 1 || !xm)
    return fail(ASR_E_UNSUPPORTED, "RK2 stack forward: needs C=64, W=32, >= 4 row bands per image");
  if (y_stride < (long)N * H * W * C) return fail(ASR_E_ARG, "RK2 stack forward: y_stride smaller than one activation");
  int cus = cu_count();
  if (cus <= 0) cus = 256;
  const int grid = std::max(1, std::min(N, 2 * cus));
  const size_t lds = 3 * (size_t)(kFwdBR + 2) * (W + 2) * C * 2;  // k_fwd3_stack's ring of three tiles
  hipLaunchKernelGGL((blk::k_fwd3_stack<64, 32, kFwdBR, true>), dim3(grid), dim3(256), lds, s, (const bf16*)x0,
                     (bf16*)ys, y_stride, masks, mask_stride, (const bf16*)w, w_stride, bias, bias_stride, h, N, H, L, 0,
                     (bf16*)xm, masks2);
  ASR_LAUNCH_CHECK("k_fwd3_stack<RK2>");
  return ASR_OK;
}

int block_bwd_mfma(int mode, const void* dy, const void* x, const uint8_t* mask, const void* w, float h,
                   float two_gamma, int N, int H, int W, int C, void* dx, float* slabs, int* nslabs, const void* extra,
                   int skip_dy, hipStream_t s, int relu_dx, int* relu_done, const float* fold_slabs, int fold_P,
                   float* fold_grp, int* fold_done, int accum) {
  if (relu_done) *relu_done = 0;
  if (fold_done) *fold_done = 0;
  if (fold_P > kMaxBlockSlabs) fold_P = 0;  // (never: slab counts are grid sizes)
  if (W != 32) return fail(ASR_E_UNSUPPORTED, "bf16 block: W=%d not supported (W must be 32)", W);
  switch (C) {
    case 16:
      return launch_bwd<16, 32>(mode, dy, x, mask, w, h, two_gamma, N, H, dx, slabs, nslabs, extra, skip_dy, relu_dx,
                                relu_done, fold_slabs, fold_P, fold_grp, fold_done, accum, s);
    case 32:
      return launch_bwd<32, 32>(mode, dy, x, mask, w, h, two_gamma, N, H, dx, slabs, nslabs, extra, skip_dy, relu_dx,
                                relu_done, fold_slabs, fold_P, fold_grp, fold_done, accum, s);
    case 64:
      return launch_bwd<64, 32>(mode, dy, x, mask, w, h, two_gamma, N, H, dx, slabs, nslabs, extra, skip_dy, relu_dx,
                                relu_done, fold_slabs, fold_P, fold_grp, fold_done, accum, s);
  }
  return fail(ASR_E_UNSUPPORTED, "bf16 block: C=%d not supported (16, 32, 64)", C);
}

}  // namespace asr

// test knob: force the stacked backward's grid (a grid larger than the
// resident capacity makes the in-launch hand-off run out and degrade to the
// post-launch reduction); 0 restores the default (one workgroup per CU)
extern "C" int asr_debug_stack_backward(int grid) {
  if (grid < 0 || grid > asr::kMaxBlockSlabs)
    return asr::fail(ASR_E_ARG, "asr_debug_stack_backward: grid must be in 0..%d", asr::kMaxBlockSlabs);
  asr::g_stack_grid_override = grid;
  return ASR_OK;
}

namespace asr {
namespace blk {
// asr_stack_status: read (and with reset, clear) the degraded-wait count in one
// device atomic, into the calling host thread's own result word
__global__ void k_stack_status_take(int reset, unsigned* out) {
  *out = reset ? __hip_atomic_exchange(&g_stack_degraded, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
               : __hip_atomic_load(&g_stack_degraded, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
}  // namespace blk
}  // namespace asr

// host, blocking: waits of stacked-backward workgroups that ran out since the
// last reset (each one a slower launch, never a wrong gradient); reset != 0
// then clears the count (atomically with the read, on the device).  Each call
// has its own result word (concurrent callers never read each other's), and
// the launch status comes from hipLaunchKernel itself: no hipGetLastError,
// which would also report and clear an unrelated pending error.
extern "C" int asr_stack_status(int reset) {
  unsigned* d = nullptr;
  if (hipMalloc(&d, sizeof(unsigned)) != hipSuccess) return asr::fail(ASR_E_HIP, "asr_stack_status: hipMalloc failed");
  int rs = reset ? 1 : 0;
  void* args[] = {&rs, &d};
  hipError_t e = hipLaunchKernel((const void*)asr::blk::k_stack_status_take, dim3(1), dim3(1), args, 0, (hipStream_t)0);
  unsigned n = 0;
  if (e == hipSuccess) e = hipMemcpy(&n, d, sizeof(n), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return asr::fail(ASR_E_HIP, "asr_stack_status: %s", hipGetErrorString(e));
  return (int)std::min<unsigned>(n, 0x7fffffffu);
}

#if ASR_STAMP_BUILD
extern "C" int asr_debug_stamps(void* host, size_t bytes) {
  if (bytes > sizeof(asr::blk::g_stamps)) bytes = sizeof(asr::blk::g_stamps);
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(asr::blk::g_stamps), bytes) == hipSuccess ? 0 : -4;
}
#endif
