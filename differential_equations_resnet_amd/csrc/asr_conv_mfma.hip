// bf16 MFMA kernels of the antisymmetric 3x3 conv / Euler block (gfx950).
//
// Reference operator: Conv2DAntisymmetric3By3.call (tf.nn.conv2d SAME NHWC +
// bias, layers/tfkeras_layer_Conv2DAntisymmetric3By3.py:157-171) inside
// single_layer_identity_block (relu, h*, +input: models/tfkeras_resnets.py:69-92)
// and its autodiff (training/training.py:300).
//
// Formulation (implicit GEMM on v_mfma_f32_16x16x32_bf16):
//   Z^T[o][p] = sum_kappa W^T[o][kappa] * X[p][kappa],  kappa = tap*C + i
// with A = W^T held in VGPRs for the whole persistent workgroup (packed by
// asr_theta_to_w so each fragment is one 16-byte load per lane), B = the
// im2col patch read straight out of an LDS image of the input band (the 3x3
// shift is only an LDS address offset), fp32 accumulation, and a fused
// epilogue.  Because A^T = -A + 2*gamma*I for the assembled W, the input
// gradient (dgrad) is the SAME kernel on dz = h*dy*mask with the SAME
// fragments, and only the epilogue changes.
//
// LDS image of a band of BR output rows: (BR+2) rows x (W+2) columns (zero
// halo) x C channels bf16, 16-byte chunks XOR-swizzled per column
// (swz(col)), chosen with tools/lds_banks.py so the B-fragment ds_read_b128
// is conflict-free.
//
// wgrad:  dW[(tap,i)][o] = sum_p X[p+s(tap)][i] * dz[p][o]  (K = pixels); both
// operands are pixel-contiguous per lane, read from the same NHWC LDS images
// with ds_read_b64_tr_b16 (hardware transpose).  Each persistent workgroup
// keeps its dW tile set in AGPR/VGPR accumulators over all of its bands and
// writes one fp32 partial slab; asr_theta.hip reduces the slabs and projects
// them onto theta.
#include "asr_common.h"

namespace asr {

enum { FWD_EULER = 0, FWD_CONV = 1, BWD_EULER = 2, BWD_CONV = 3 };

template <int C>
struct Geo {
  static constexpr int NQ = C / 8;              // 16-byte chunks per pixel
  static constexpr int OT = C / 16;             // 16-channel tiles
  static constexpr int KS = (9 * C + 31) / 32;  // 32-deep k-steps
  static constexpr int OSPLIT = (C == 64) ? 2 : 1;
  static constexpr int OTW = OT / OSPLIT;  // o-tiles per wave (fwd/dgrad)
  static constexpr int RSPLIT = 4 / OSPLIT;
  // wgrad decomposition: m-tiles (16 rows of 9C) per wave = 9
  static constexpr int MT = 9 * C / 16;
  static constexpr int MTW = 9;
  static constexpr int TG = MT / MTW;   // tile groups
  static constexpr int KSPLIT = 4 / TG; // waves splitting K inside a tile group
  __device__ __forceinline__ static int swz(int col) {
    if constexpr (C == 64) return col & 7;
    else if constexpr (C == 32) return (col >> 1) & 3;
    else return 0;
  }
};

template <int C>
__device__ __forceinline__ int tile_off(int row, int col, int q, int TW) {
  return ((row * TW + col) * Geo<C>::NQ + (q ^ Geo<C>::swz(col))) * 16;
}

__device__ __forceinline__ uint4 u4zero() { return make_uint4(0, 0, 0, 0); }

// Mask layout (asr.h asr_mask_bytes): bit (pixel*C + o), pixel = (n*H + y)*W + x,
// i.e. NHWC bit order; one byte = 8 channels of one pixel = one 16-byte chunk.
// dz = h*dy*mask for the chunk of 8 channels whose mask byte is mb.
__device__ __forceinline__ uint4 dz_chunk(uint4 dyv, unsigned mb, float h, float* dzf) {
  const bf16x8 dy8 = *(const bf16x8*)&dyv;
  bf16x8 out;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float d = ((mb >> j) & 1u) ? h * (float)dy8[j] : 0.f;
    dzf[j] = d;
    out[j] = (bf16)d;
  }
  return *(const uint4*)&out;
}

// Stage rows [y0-1, y0+rows] x cols [-1, W] of `src` (bf16 NHWC) into an LDS
// tile (zero outside the image).  All global loads of a batch are issued
// before any LDS store so their latencies overlap.
template <int C, int W, int MAXROWS, int KB = 4>
__device__ __forceinline__ void stage_plain(const bf16* __restrict__ src, unsigned char* tile, int n, int y0,
                                            int rows, int H, int tid) {
  constexpr int TW = W + 2, NQ = C / 8;
  const int nch = rows * TW * NQ;
  for (int base = 0; base < nch; base += 256 * KB) {
    uint4 v[KB];
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      const int c = base + tid + 256 * k;
      v[k] = u4zero();
      const int q = c % NQ, pc = c / NQ, col = pc % TW, r = pc / TW;
      const int gy = y0 + r, gx = col - 1;
      if (c < nch && gy >= 0 && gy < H && gx >= 0 && gx < W)
        v[k] = *(const uint4*)(src + (((long)n * H + gy) * W + gx) * C + q * 8);
    }
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      const int c = base + tid + 256 * k;
      const int q = c % NQ, pc = c / NQ, col = pc % TW, r = pc / TW;
      if (c < nch) *(uint4*)(tile + tile_off<C>(r, col, q, TW)) = v[k];
    }
  }
}

// Stage dz = h*dy*mask (EULER) or dy (CONV) for rows [y0+r0, y0+r0+rows) into
// `tz` (tile rows 0..rows-1) and optionally the raw dy into `ty` (same rows,
// shifted by ty_row).  Accumulates db partial sums (8 channels per thread).
template <int C, int W, int MAXROWS, bool EULER, int KB = 4>
__device__ __forceinline__ void stage_dz(const bf16* __restrict__ dy, const uint8_t* __restrict__ mask,
                                         unsigned char* tz, unsigned char* ty, int ty_lo, int ty_hi, int n,
                                         int gy0, int rows, int H, float h, int tid, float* dbacc, int db_lo,
                                         int db_hi) {
  constexpr int TW = W + 2, NQ = C / 8;
  const int nch = rows * TW * NQ;
  for (int base = 0; base < nch; base += 256 * KB) {
    uint4 v[KB];
    unsigned mb[KB];
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      const int c = base + tid + 256 * k;
      v[k] = u4zero();
      mb[k] = 0;
      const int q = c % NQ, pc = c / NQ, col = pc % TW, r = pc / TW;
      const int gy = gy0 + r, gx = col - 1;
      if (c < nch && gy >= 0 && gy < H && gx >= 0 && gx < W) {
        const long pix = ((long)n * H + gy) * W + gx;
        v[k] = *(const uint4*)(dy + pix * C + q * 8);
        if constexpr (EULER) mb[k] = mask[pix * NQ + q];
      }
    }
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      const int c = base + tid + 256 * k;
      const int q = c % NQ, pc = c / NQ, col = pc % TW, r = pc / TW;
      if (c < nch) {
        float f[8];
        uint4 dz;
        if constexpr (EULER) {
          dz = dz_chunk(v[k], mb[k], h, f);
        } else {
          dz = v[k];
          const bf16x8 d8 = *(const bf16x8*)&v[k];
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = (float)d8[j];
        }
        *(uint4*)(tz + tile_off<C>(r, col, q, TW)) = dz;
        if (ty && r >= ty_lo && r < ty_hi) *(uint4*)(ty + tile_off<C>(r - ty_lo, col, q, TW)) = v[k];
        if (dbacc && r >= db_lo && r < db_hi) {
#pragma unroll
          for (int j = 0; j < 8; ++j) dbacc[j] += f[j];
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// forward conv / Euler step, and dgrad (MODE >= BWD_EULER)
// ---------------------------------------------------------------------------
template <int C, int W, int BR, int MODE>
__global__ __launch_bounds__(256, 2) void k_conv_mfma(const bf16* __restrict__ xin, bf16* __restrict__ out,
                                                      uint8_t* __restrict__ mask, const bf16* __restrict__ wpack,
                                                      const float* __restrict__ bias, float h, float two_gamma,
                                                      int N, int H) {
  using G = Geo<C>;
  constexpr int TW = W + 2, PT = W / 16, NQ = G::NQ, OTW = G::OTW, KS = G::KS;
  constexpr bool BWD = MODE >= BWD_EULER;
  constexpr bool EULER = (MODE == FWD_EULER) || (MODE == BWD_EULER);
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  unsigned char* tileA = lds;                          // x (fwd) or dz (bwd), with halo
  unsigned char* tileB = lds + (BR + 2) * TW * NQ * 16;  // bwd: dy, interior rows

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int oh = wave % G::OSPLIT, rg = wave / G::OSPLIT;
  const int g = lane >> 4, lx = lane & 15;

  // W^T fragments of this wave's o-tiles, resident for the whole kernel
  bf16x8 A[OTW][KS];
#pragma unroll
  for (int t = 0; t < OTW; ++t)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      A[t][ks] = *(const bf16x8*)(wpack + (((long)(oh * OTW + t) * KS + ks) * 64 + lane) * 8);

  // per-lane B-fragment LDS offsets for every k-step (row 0, pixel tile 0)
  int boff[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    int tap = (32 * ks + 8 * g) / C;
    if (tap > 8) tap = 8;  // C=16 tail: A is zero there
    const int q = ((32 * ks + 8 * g) % C) / 8;
    const int ky = tap / 3, kx = tap % 3;
    boff[ks] = tile_off<C>(ky, lx + kx, q, TW);
  }

  float bz[OTW][4];
#pragma unroll
  for (int t = 0; t < OTW; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) bz[t][e] = (!BWD && bias) ? bias[16 * (oh * OTW + t) + 4 * g + e] : 0.f;

  const int nb = (H + BR - 1) / BR;
  const long items = (long)N * nb;
  for (long item = blockIdx.x; item < items; item += gridDim.x) {
    const int n = (int)(item / nb);
    const int y0 = (int)(item % nb) * BR;
    const int rows = min(BR, H - y0);
    // ---- stage the band (+halo) into LDS ----
    if constexpr (BWD)
      stage_dz<C, W, BR + 2, EULER>(xin, mask, tileA, tileB, 1, rows + 1, n, y0 - 1, rows + 2, H, h, tid, nullptr, 0,
                                    0);
    else
      stage_plain<C, W, BR + 2>(xin, tileA, n, y0 - 1, rows + 2, H, tid);
    __syncthreads();

    // ---- implicit GEMM + epilogue, one output row at a time ----
    for (int r = rg; r < rows; r += G::RSPLIT) {
      f32x4 acc[OTW][PT];
#pragma unroll
      for (int t = 0; t < OTW; ++t)
#pragma unroll
        for (int pt = 0; pt < PT; ++pt) acc[t][pt] = f32x4{0.f, 0.f, 0.f, 0.f};
      const unsigned char* rowbase = tileA + r * TW * NQ * 16;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
        for (int pt = 0; pt < PT; ++pt) {
          const bf16x8 B = *(const bf16x8*)(rowbase + boff[ks] + pt * 16 * NQ * 16);
#pragma unroll
          for (int t = 0; t < OTW; ++t)
            acc[t][pt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[t][ks], B, acc[t][pt], 0, 0, 0);
        }
      }
      const int gy = y0 + r;
#pragma unroll
      for (int pt = 0; pt < PT; ++pt) {
        const int px = 16 * pt + lx;
        unsigned mword = 0;  // FWD_EULER: relu bits of this pixel's OTW*16 channels
#pragma unroll
        for (int t = 0; t < OTW; ++t) {
          const int o0 = 16 * (oh * OTW + t) + 4 * g;
          const int co = tile_off<C>(r + 1, px + 1, o0 >> 3, TW) + (o0 & 4) * 2;
          float v[4];
          if constexpr (MODE == FWD_EULER) {
            const bf16x4 xr = *(const bf16x4*)(tileA + co);
            unsigned nib = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float z = acc[t][pt][e] + bz[t][e];
              nib |= (z > 0.f ? 1u : 0u) << e;
              v[e] = (float)xr[e] + h * fmaxf(z, 0.f);
            }
            mword |= nib << (16 * t + 4 * g);
          } else if constexpr (MODE == FWD_CONV) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = acc[t][pt][e] + bz[t][e];
          } else {
            const bf16x4 dzr = *(const bf16x4*)(tileA + co);
            const int cob = tile_off<C>(r, px + 1, o0 >> 3, TW) + (o0 & 4) * 2;
            const bf16x4 dyr = *(const bf16x4*)(tileB + cob);
#pragma unroll
            for (int e = 0; e < 4; ++e)
              v[e] = (EULER ? (float)dyr[e] : 0.f) - acc[t][pt][e] + two_gamma * (float)dzr[e];
          }
          bf16x4 o4;
#pragma unroll
          for (int e = 0; e < 4; ++e) o4[e] = (bf16)v[e];
          *(bf16x4*)(out + (((long)n * H + gy) * W + px) * C + o0) = o4;
        }
        if constexpr (MODE == FWD_EULER) {
          // gather the 4 lane groups' nibbles: lanes lx, lx+16, lx+32, lx+48 share the pixel
          mword |= __shfl_xor(mword, 16);
          mword |= __shfl_xor(mword, 32);
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
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// wgrad: per-workgroup fp32 partial of dW and db
// ---------------------------------------------------------------------------
__device__ __forceinline__ bf16x8 tr_pair(const unsigned char* p0, const unsigned char* p1) {
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((ASR_LDS s16x4*)p0);
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((ASR_LDS s16x4*)p1);
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 c = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return *(bf16x8*)&c;
}

template <int C, int W, int BR, int MODE>
__global__ __launch_bounds__(256, 2) void k_wgrad_mfma(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                       const uint8_t* __restrict__ mask, float h, int N, int H,
                                                       float* __restrict__ slabs) {
  using G = Geo<C>;
  constexpr int TW = W + 2, NQ = G::NQ, OT = G::OT, MTW = G::MTW;
  constexpr int KPR = W / 32;  // 32-pixel k-steps per image row
  constexpr bool EULER = (MODE == BWD_EULER);
  static_assert(W % 32 == 0, "wgrad k-steps are 32 pixels of one row");
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  unsigned char* tileX = lds;
  unsigned char* tileZ = lds + (BR + 2) * TW * NQ * 16;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tg = wave % G::TG, kg = wave / G::TG;
  const int g = lane >> 4, lx = lane & 15;
  const int tq = lx >> 2, tp = lx & 3;  // lane 4*tq+tp of its 16-lane group (tr read)

  f32x4 acc[MTW][OT];
#pragma unroll
  for (int mi = 0; mi < MTW; ++mi)
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) acc[mi][ot] = f32x4{0.f, 0.f, 0.f, 0.f};

  float dbacc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) dbacc[j] = 0.f;

  const int nb = (H + BR - 1) / BR;
  const long items = (long)N * nb;
  for (long item = blockIdx.x; item < items; item += gridDim.x) {
    const int n = (int)(item / nb);
    const int y0 = (int)(item % nb) * BR;
    const int rows = min(BR, H - y0);
    stage_plain<C, W, BR + 2>(x, tileX, n, y0 - 1, rows + 2, H, tid);
    stage_dz<C, W, BR, EULER>(dy, mask, tileZ, nullptr, 0, 0, n, y0, rows, H, h, tid, dbacc, 0, BR);
    __syncthreads();

    for (int kk = kg; kk < rows * KPR; kk += G::KSPLIT) {
      const int r = kk / KPR, kb = kk % KPR;
      const int pb = 32 * kb + 8 * g + tq;  // pixel of this lane's tr-read row (first half)
      bf16x8 Bf[OT];
#pragma unroll
      for (int ot = 0; ot < OT; ++ot) {
        const int q = 2 * ot + (tp >> 1);
        const unsigned char* p0 = tileZ + tile_off<C>(r, pb + 1, q, TW) + 8 * (tp & 1);
        const unsigned char* p1 = tileZ + tile_off<C>(r, pb + 5, q, TW) + 8 * (tp & 1);
        Bf[ot] = tr_pair(p0, p1);
      }
#pragma unroll
      for (int mi = 0; mi < MTW; ++mi) {
        const int mt = tg * MTW + mi;
        const int tap = (16 * mt) / C, it = ((16 * mt) % C) / 16;
        const int ky = tap / 3, kx = tap % 3;
        const int q = 2 * it + (tp >> 1);
        const unsigned char* p0 = tileX + tile_off<C>(r + ky, pb + kx, q, TW) + 8 * (tp & 1);
        const unsigned char* p1 = tileX + tile_off<C>(r + ky, pb + 4 + kx, q, TW) + 8 * (tp & 1);
        const bf16x8 Af = tr_pair(p0, p1);
#pragma unroll
        for (int ot = 0; ot < OT; ++ot) acc[mi][ot] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Af, Bf[ot], acc[mi][ot], 0, 0, 0);
      }
    }
    __syncthreads();
  }

  // ---- K-split reduction inside the workgroup (C < 64) ----
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
  }
  float* slab = slabs + (long)blockIdx.x * (9 * C * C + C);
  if (kg == 0) {
#pragma unroll
    for (int mi = 0; mi < MTW; ++mi)
#pragma unroll
      for (int ot = 0; ot < OT; ++ot)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int m = 16 * (tg * MTW + mi) + 4 * g + e;
          slab[(long)m * C + 16 * ot + lx] = acc[mi][ot][e];
        }
  }
  // ---- db: threads with equal (tid % NQ) own the same 8 channels ----
  __syncthreads();
  float* dbl = (float*)lds;
#pragma unroll
  for (int j = 0; j < 8; ++j) dbl[j * 256 + tid] = dbacc[j];
  __syncthreads();
  if (tid < C) {
    const int q = tid / 8, j = tid % 8;
    float s = 0.f;
    for (int t = q; t < 256; t += NQ) s += dbl[j * 256 + t];
    slab[9 * C * C + tid] = s;
  }
}

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
constexpr int kMaxSlabs = 512;

constexpr int kBR = 8;  // output rows per band (work item)

template <int C, int W>
static size_t conv_lds(int BR, bool bwd) {
  size_t t = (size_t)(BR + 2) * (W + 2) * (C / 8) * 16;
  if (bwd) t += (size_t)BR * (W + 2) * (C / 8) * 16;
  return t;
}

template <int C, int W>
static size_t wgrad_lds(int BR) {
  size_t t = (size_t)(BR + 2) * (W + 2) * (C / 8) * 16 + (size_t)BR * (W + 2) * (C / 8) * 16;
  using G = Geo<C>;
  size_t red = (size_t)(G::KSPLIT - 1) * G::TG * G::MTW * G::OT * 256 * 4;
  size_t dbl = 8 * 256 * 4;
  return std::max(t, std::max(red, dbl));
}

static int grid_for(long items) {
  int cus = cu_count();
  if (cus <= 0) cus = 256;
  long g = std::min<long>(items, 2L * cus);
  g = std::min<long>(g, kMaxSlabs);
  return (int)std::max<long>(g, 1);
}

template <int C, int W>
static int launch_conv_mfma(int mode, const void* xin, void* out, uint8_t* mask, const void* w, const float* bias,
                            float h, float two_gamma, int N, int H, hipStream_t s) {
  const int BR = kBR;
  const long items = (long)N * ((H + BR - 1) / BR);
  const int grid = grid_for(items);
  const bool bwd = mode >= BWD_EULER;
  const size_t lds = conv_lds<C, W>(BR, bwd);
#define ASR_CONV_CASE(M)                                                                                   \
  case M:                                                                                                  \
    hipLaunchKernelGGL((k_conv_mfma<C, W, kBR, M>), dim3(grid), dim3(256), lds, s, (const bf16*)xin,        \
                       (bf16*)out, mask, (const bf16*)w, bias, h, two_gamma, N, H);                        \
    break;
  switch (mode) {
    ASR_CONV_CASE(FWD_EULER)
    ASR_CONV_CASE(FWD_CONV)
    ASR_CONV_CASE(BWD_EULER)
    ASR_CONV_CASE(BWD_CONV)
    default:
      return fail(ASR_E_ARG, "bad conv mode");
  }
#undef ASR_CONV_CASE
  ASR_LAUNCH_CHECK("k_conv_mfma");
  return ASR_OK;
}

template <int C, int W>
static int launch_wgrad_mfma(int mode, const void* x, const void* dy, const uint8_t* mask, float h, int N, int H,
                             float* slabs, int* nslabs, hipStream_t s) {
  const int BR = kBR;
  const long items = (long)N * ((H + BR - 1) / BR);
  const int grid = grid_for(items);
  *nslabs = grid;
  const size_t lds = wgrad_lds<C, W>(BR);
  if (mode == BWD_EULER)
    hipLaunchKernelGGL((k_wgrad_mfma<C, W, kBR, BWD_EULER>), dim3(grid), dim3(256), lds, s, (const bf16*)x,
                       (const bf16*)dy, mask, h, N, H, slabs);
  else
    hipLaunchKernelGGL((k_wgrad_mfma<C, W, kBR, BWD_CONV>), dim3(grid), dim3(256), lds, s, (const bf16*)x,
                       (const bf16*)dy, mask, h, N, H, slabs);
  ASR_LAUNCH_CHECK("k_wgrad_mfma");
  return ASR_OK;
}

bool mfma_supported(int C, int W) { return (C == 16 || C == 32 || C == 64) && W == 32; }

int conv_mfma(int mode, const void* xin, void* out, uint8_t* mask, const void* w, const float* bias, float h,
              float two_gamma, int N, int H, int W, int C, hipStream_t s) {
  if (W != 32) return fail(ASR_E_UNSUPPORTED, "bf16 conv: W=%d not supported (W must be 32)", W);
  switch (C) {
    case 16: return launch_conv_mfma<16, 32>(mode, xin, out, mask, w, bias, h, two_gamma, N, H, s);
    case 32: return launch_conv_mfma<32, 32>(mode, xin, out, mask, w, bias, h, two_gamma, N, H, s);
    case 64: return launch_conv_mfma<64, 32>(mode, xin, out, mask, w, bias, h, two_gamma, N, H, s);
  }
  return fail(ASR_E_UNSUPPORTED, "bf16 conv: C=%d not supported (16, 32, 64)", C);
}

int wgrad_mfma(int mode, const void* x, const void* dy, const uint8_t* mask, float h, int N, int H, int W, int C,
               float* slabs, int* nslabs, hipStream_t s) {
  if (W != 32) return fail(ASR_E_UNSUPPORTED, "bf16 wgrad: W=%d not supported", W);
  switch (C) {
    case 16: return launch_wgrad_mfma<16, 32>(mode, x, dy, mask, h, N, H, slabs, nslabs, s);
    case 32: return launch_wgrad_mfma<32, 32>(mode, x, dy, mask, h, N, H, slabs, nslabs, s);
    case 64: return launch_wgrad_mfma<64, 32>(mode, x, dy, mask, h, N, H, slabs, nslabs, s);
  }
  return fail(ASR_E_UNSUPPORTED, "bf16 wgrad: C=%d not supported", C);
}

}  // namespace asr
