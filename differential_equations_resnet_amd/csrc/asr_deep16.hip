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
// Conv = implicit GEMM on v_mfma_f32_16x16x32_bf16, kappa = tap*16 + i:
//   Z^T[o][p] = b[o] + sum_kappa W^T[o][kappa] X[p][kappa]
// A = W^T (16 x 144, padded to 5 k-steps of 32) in VGPRs per layer; B read
// from the LDS image: lane (pixel lx, group g) of k-step ks reads the 16-B
// chunk (g & 1) of tap 2ks + (g >> 1) at pixel lx, one ds_read_b128 (the
// NHWC 32-B pixels are bank-conflict-free for the b128 lane groups).  The
// padded tap 9 re-reads tap 8 (finite data, multiplied by A = 0).
// Same accumulation order as the per-block kernel (bias, then k-steps 0..4),
// so a layer's result is bitwise that of k_fwd<16,...>.
#include <type_traits>

#include "asr_common.h"
#include "asr_device.h"

namespace asr {
namespace deep {

using namespace blk;

constexpr int C = 16, W = 32, H = 32, TW = W + 2;
constexpr int ROWB = TW * C * 2;       // 1088 B per tile row (halo columns included)
constexpr int TILE = (H + 2) * ROWB;   // 36992 B per image tile (halo rows included)
constexpr int KS = 5;                  // k-steps of 32 over kappa = 9 taps x 16 channels (+ pad)
constexpr int WSTRIDE = KS * 512;      // packed W^T elements per layer (asr_wpack_elems(16))
constexpr int NWAVE = 4;               // waves per workgroup; wave w owns image rows [8w, 8w+8)
constexpr int RPW = H / NWAVE;

__device__ __forceinline__ void load_wt(const bf16* __restrict__ w, int lane, bf16x8 (&A)[KS]) {
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) A[ks] = *(const bf16x8*)(w + (ks * 64 + lane) * 8);
}

// zero the whole tile (halo included); interiors are overwritten later
__device__ __forceinline__ void zero_tile(unsigned char* t, int tid, int nt) {
  for (int i = tid; i < TILE / 16; i += nt) ((uint4*)t)[i] = make_uint4(0, 0, 0, 0);
}

// x_{l+1} for l = 0 .. L-1 of every image the workgroup owns.
//   x0:    [N,32,32,16] bf16 (the stem output)
//   y0:    output of layer 0; layer l writes y0 + l*y_stride (store_all), or
//          only layer L-1 writes y0 (inference)
//   mask0: relu masks, layer l at mask0 + l*mask_stride bytes (may be null)
//   wpack: packed W^T, layer l at wpack + l*WSTRIDE; bias: layer l at bias + l*bias_stride
template <bool STORE_ALL>
__global__ __launch_bounds__(64 * NWAVE, 2) void k_fwd16_fused(const bf16* __restrict__ x0, bf16* __restrict__ y0,
                                                            long y_stride, uint8_t* __restrict__ mask0,
                                                            long mask_stride, const bf16* __restrict__ wpack,
                                                            const float* __restrict__ bias, long bias_stride,
                                                            float h, int N, int L) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, lx = lane & 15;
  const int r0 = wave * RPW;
  zero_tile(lds, tid, 64 * NWAVE);
  zero_tile(lds + TILE, tid, 64 * NWAVE);
  // per-lane B offsets of the 5 k-steps relative to (output row, pixel tile)
  unsigned boff[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int tap = min(2 * ks + (g >> 1), 8);
    boff[ks] = (unsigned)(((tap / 3) * TW + tap % 3 + lx) * 32 + (g & 1) * 16);
  }
  // residual / output offset of the lane's 4 channels 4g..4g+3 of pixel lx
  const unsigned xoff = (unsigned)((TW + 1 + lx) * 32 + 8 * g);
  __syncthreads();

  for (int n = blockIdx.x; n < N; n += gridDim.x) {
    // stage x0 of image n in tile 0 (interiors: one 1 KiB DMA per image row)
    {
      const unsigned char* src = (const unsigned char*)(x0 + (long)n * H * W * C);
#pragma unroll
      for (int k = 0; k < RPW; ++k) {
        const int r = r0 + k;
        dma16(src + r * 1024 + lane * 16, lds + (r + 1) * ROWB + 32);
      }
    }
    bf16x8 A[KS], An[KS];
    load_wt(wpack, lane, A);
    float bz[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) bz[e] = bias ? bias[4 * g + e] : 0.f;
    barrier_vm(0);  // the image's rows landed in every wave's share

    for (int l = 0; l < L; ++l) {
      const unsigned char* src = lds + (l & 1) * TILE;
      unsigned char* dst = lds + ((l + 1) & 1) * TILE;
      const bool more = l + 1 < L;
      float bn[4];
      if (more) {  // next layer's W^T fragments and bias (L2-resident) while this one runs
        load_wt(wpack + (long)(l + 1) * WSTRIDE, lane, An);
#pragma unroll
        for (int e = 0; e < 4; ++e) bn[e] = bias ? bias[(l + 1) * bias_stride + 4 * g + e] : 0.f;
      }
      const bool store = STORE_ALL || l == L - 1;
      bf16* yl = y0 + (STORE_ALL ? (long)l * y_stride : 0) + (long)n * H * W * C;
      uint8_t* ml = mask0 ? mask0 + (long)l * mask_stride + (long)n * H * W * (C / 8) : nullptr;
#pragma unroll
      for (int k = 0; k < RPW; ++k) {
        const int r = r0 + k;
        unsigned mw[2];
#pragma unroll
        for (int pt = 0; pt < 2; ++pt) {
          const unsigned char* tb = src + r * ROWB + pt * 512;
          f32x4 acc = {bz[0], bz[1], bz[2], bz[3]};
          bf16x8 B[KS];
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) B[ks] = *(const bf16x8*)(tb + boff[ks]);
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[ks], B[ks], acc, 0, 0, 0);
          // epilogue: y = x + h * relu(z) (fp32, one rounding), relu bits
          const bf16x4 xr = *(const bf16x4*)(tb + xoff);
          bf16x4 o4;
          unsigned nib = 0;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float z = acc[e];
            const bool pos = z > 0.f;  // relu'(z) as TF's ReluGrad: z > 0
            nib |= (pos ? 1u : 0u) << e;
            const float rz = __builtin_bit_cast(float, __builtin_bit_cast(unsigned, z) & (pos ? ~0u : 0u));
            o4[e] = (bf16)fmaf(h, rz, (float)xr[e]);
          }
          *(bf16x4*)(dst + r * ROWB + pt * 512 + xoff) = o4;
          if (store) *(bf16x4*)(yl + ((r * W) + 16 * pt + lx) * C + 4 * g) = o4;
          // the pixel's 16 channel bits: OR over the four lane groups g
          unsigned m = nib << (4 * g);
          const auto s16 = __builtin_amdgcn_permlane16_swap(m, m, false, false);
          m = s16[0] | s16[1];
          const auto s32 = __builtin_amdgcn_permlane32_swap(m, m, false, false);
          mw[pt] = s32[0] | s32[1];
        }
        // row r's 32 mask words (64 B): lanes 0-15 pixel tile 0, 16-31 tile 1
        if (ml && lane < 32) *(uint16_t*)(ml + (r * W + lane) * 2) = (uint16_t)(lane < 16 ? mw[0] : mw[1]);
      }
      if (more) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) A[ks] = An[ks];
#pragma unroll
        for (int e = 0; e < 4; ++e) bz[e] = bn[e];
      }
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
// with dx kept in LDS across layers (no HBM round trip per block).  The
// layers run in segments of KSEG: the weight gradients of a segment's layers
// accumulate in registers over all images of the workgroup, so each layer
// gets ONE slab [dW (9*16*16) | db (16)] fp32 per workgroup (the layout
// asr_api's reduce_slabs_to_groups / project_layers consume), and dx crosses
// HBM only at segment boundaries.  x_{l-1} and mask_{l-1} are DMA'd into the
// second buffers while layer l computes.
//
// dgrad: the forward's implicit GEMM with dzm in place of x (bitwise the
// per-block kernel's dx).  wgrad: GEMM with M = tap-channel (16 per m-tile:
// one tap), N = o, K = pixels (one image row of 32 per k-step); both operands
// by ds_read_b64_tr_b16 (T10) from the x tile (shifted by the tap) and the dz
// tile.  The 8 k-rows of lane group g are pixels 8g + 4*(hh ^ (g & 1)) + q for
// the two reads hh: the halves of odd groups are swapped so the two 16-lane
// groups of each 32-lane half read disjoint banks.
// LDS: dx (32 KiB) | dz tile | 2 x tiles | 2 x 2 KiB masks | 4 KiB mask table.
// ---------------------------------------------------------------------------
constexpr int KSEG = 6;                  // layers per segment (dW accumulators in registers)
constexpr int ES = 9 * C * C + C;        // slab floats per layer
constexpr int DXB = H * W * C * 2;       // 32 KiB
constexpr int MB = H * W * C / 8;        // 2 KiB of relu bits per image
constexpr int L_DX = 0, L_DZ = L_DX + DXB, L_X = L_DZ + TILE, L_M = L_X + 2 * TILE, L_TAB = L_M + 2 * MB;
constexpr int L_TOTAL = L_TAB + 4096;
static_assert(L_TOTAL <= 160 * 1024, "LDS budget");
static_assert(4 * 9 * 4 * 64 * 4 + 4 * C * 4 <= 2 * TILE, "segment-end reduction area");

__device__ __forceinline__ bf16x8 tr2(const unsigned char* base, unsigned o0, unsigned o1) {
  return tr_pair(base + o0, base + o1);
}

__global__ __launch_bounds__(64 * NWAVE, 1) void k_bwd16_fused(bf16* __restrict__ dbufA, bf16* __restrict__ dbufB,
                                                              const bf16* __restrict__ xs, long x_stride,
                                                              const uint8_t* __restrict__ masks, long mask_stride,
                                                              const bf16* __restrict__ wpack, float h, float two_gamma,
                                                              int N, int L, float* __restrict__ slabs, int PS) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, lx = lane & 15, q = lx >> 2, p = lx & 3;
  const int r0 = wave * RPW;
  const int P = gridDim.x, b = blockIdx.x;
  const float hs2g = h * two_gamma;
  // zero the dz tile and both x tiles (halo rows / columns stay zero), build the mask table
  for (int i = tid; i < 3 * TILE / 16; i += 64 * NWAVE) ((uint4*)(lds + L_DZ))[i] = make_uint4(0, 0, 0, 0);
  {
    unsigned* tab = (unsigned*)(lds + L_TAB);  // dword d of byte m: 0xffff per set bit of (m >> 2d) & 3
    for (int i = tid; i < 1024; i += 64 * NWAVE) {
      const unsigned m = (unsigned)i >> 2, d = (unsigned)i & 3;
      tab[i] = (((m >> (2 * d)) & 1u) ? 0xffffu : 0u) | (((m >> (2 * d + 1)) & 1u) ? 0xffff0000u : 0u);
    }
  }
  unsigned boff[KS];  // dgrad B (dz tile), as the forward
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int tap = min(2 * ks + (g >> 1), 8);
    boff[ks] = (unsigned)(((tap / 3) * TW + tap % 3 + lx) * 32 + (g & 1) * 16);
  }
  const unsigned zoff = (unsigned)((TW + 1 + lx) * 32 + 8 * g);  // dz interior value of the D layout
  const unsigned doff = (unsigned)(lx * 32 + 8 * g);              // dx (no halo) of the D layout
  unsigned toff2[2];  // wgrad tr-read lane offsets (pixel 8g + 4*(hh ^ (g&1)) + q, channels 4p..4p+3)
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) toff2[hh] = (unsigned)((8 * g + 4 * (hh ^ (g & 1)) + q) * 32 + 8 * p);
  __syncthreads();

  f32x4 acc[KSEG][9];
  float dbacc[KSEG][4];
  const int nseg = (L + KSEG - 1) / KSEG;
  for (int sg = 0; sg < nseg; ++sg) {
    const int ltop = L - 1 - sg * KSEG, kcount = min(KSEG, ltop + 1);
    const bf16* din = (sg & 1) ? dbufB : dbufA;
    bf16* dout = (sg & 1) ? dbufA : dbufB;
#pragma unroll
    for (int k = 0; k < KSEG; ++k) {
#pragma unroll
      for (int t = 0; t < 9; ++t) acc[k][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int e = 0; e < 4; ++e) dbacc[k][e] = 0.f;
    }
    for (int n = b; n < N; n += P) {
      const long img = (long)n * H * W * C;
      // stage dx at the segment top, x_ltop and mask_ltop
      {
        const unsigned char* ds = (const unsigned char*)(din + img);
        const unsigned char* xsrc = (const unsigned char*)(xs + ltop * x_stride + img);
#pragma unroll
        for (int k = 0; k < RPW; ++k) {
          const int r = r0 + k;
          dma16(ds + r * 1024 + lane * 16, lds + L_DX + r * 1024);
          dma16(xsrc + r * 1024 + lane * 16, lds + L_X + (r + 1) * ROWB + 32);
        }
        if (wave < 2) dma16(masks + ltop * mask_stride + (long)n * MB + wave * 1024 + lane * 16, lds + L_M + wave * 1024);
      }
      bf16x8 A[KS], An[KS];
      load_wt(wpack + (long)ltop * WSTRIDE, lane, A);
      barrier_vm(0);
#pragma unroll
      for (int k = 0; k < KSEG; ++k) {
        if (k >= kcount) break;
        const int l = ltop - k, cur = k & 1;
        const bool more = k + 1 < kcount;
        unsigned char* xt = lds + L_X + cur * TILE;
        const unsigned char* mt = lds + L_M + cur * MB;
        if (more) {  // x_{l-1}, mask_{l-1} into the other buffers; W of layer l-1
          const unsigned char* xsrc = (const unsigned char*)(xs + (l - 1) * x_stride + img);
#pragma unroll
          for (int kk = 0; kk < RPW; ++kk) {
            const int r = r0 + kk;
            dma16(xsrc + r * 1024 + lane * 16, lds + L_X + (cur ^ 1) * TILE + (r + 1) * ROWB + 32);
          }
          if (wave < 2)
            dma16(masks + (l - 1) * mask_stride + (long)n * MB + wave * 1024 + lane * 16,
                  lds + L_M + (cur ^ 1) * MB + wave * 1024);
          load_wt(wpack + (long)(l - 1) * WSTRIDE, lane, An);
        }
        // phase 1: dzm = dx & mask for the wave's rows (16-B chunks)
#pragma unroll 2
        for (int j = 0; j < RPW; ++j) {
          const int r = r0 + j, px = lane >> 1, hc = lane & 1;
          const unsigned char* dsrc = lds + L_DX + (r * W + px) * 32 + hc * 16;
          const uint4 dv = *(const uint4*)dsrc;
          const unsigned mb = mt[(r * W + px) * 2 + hc];
          const uint4 mv = *(const uint4*)(lds + L_TAB + mb * 16);
          *(uint4*)(lds + L_DZ + ((r + 1) * TW + px + 1) * 32 + hc * 16) =
              make_uint4(dv.x & mv.x, dv.y & mv.y, dv.z & mv.z, dv.w & mv.w);
        }
        barrier_lds();  // dz complete (the prefetch DMA keeps flying)
        // phase 2a: dgrad over the wave's rows, dx updated in place, db
#pragma unroll 1
        for (int j = 0; j < RPW; ++j) {
          const int r = r0 + j;
#pragma unroll
          for (int pt = 0; pt < 2; ++pt) {
            const unsigned char* tb = lds + L_DZ + r * ROWB + pt * 512;
            bf16x8 B[KS];
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) B[ks] = *(const bf16x8*)(tb + boff[ks]);
            f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[ks], B[ks], c, 0, 0, 0);
            const bf16x4 zr = *(const bf16x4*)(tb + zoff);
            unsigned char* dxp = lds + L_DX + (r * W + 16 * pt) * 32 + doff;
            const bf16x4 dr = *(const bf16x4*)dxp;
            bf16x4 o4;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float zf = (float)zr[e];
              dbacc[k][e] += zf;
              const float v = fmaf(-h, c[e], (float)dr[e]);
              o4[e] = (bf16)(hs2g != 0.f ? fmaf(hs2g, zf, v) : v);
            }
            *(bf16x4*)dxp = o4;
          }
        }
        // phase 2b: wgrad over the wave's rows (one k-step of 32 pixels per row)
#pragma unroll 1
        for (int j = 0; j < RPW; ++j) {
          const int r = r0 + j;
          const unsigned char* zrow = lds + L_DZ + (r + 1) * ROWB + 32;  // interior pixel 0 of row r
          const bf16x8 Bz = tr2(zrow, toff2[0], toff2[1]);
#pragma unroll
          for (int tap = 0; tap < 9; ++tap) {
            const unsigned char* xrow = xt + (r + tap / 3) * ROWB + (tap % 3) * 32;
            const bf16x8 Ax = tr2(xrow, toff2[0], toff2[1]);
            acc[k][tap] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ax, Bz, acc[k][tap], 0, 0, 0);
          }
        }
        if (more) {
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) A[ks] = An[ks];
        }
        barrier_vm(0);  // dx updated, dz and x_l consumed; x_{l-1} / mask_{l-1} landed
      }
      // dx at the segment bottom -> HBM (the next segment's input, or dx_0)
      {
        unsigned char* dst = (unsigned char*)(dout + img);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int o = (tid + j * 64 * NWAVE) * 16;
          *(uint4*)(dst + o) = *(const uint4*)(lds + L_DX + o);
        }
      }
      barrier_lds();  // dx read out before the next image's DMA overwrites it
    }
    // segment end: one slab per layer (the four waves' partials summed in a fixed order)
    float* red = (float*)(lds + L_X);
    float* dbr = red + 4 * 9 * 4 * 64;
#pragma unroll
    for (int k = 0; k < KSEG; ++k) {
      if (k >= kcount) break;
      const int l = ltop - k;
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int e = 0; e < 4; ++e) red[((wave * 9 + t) * 4 + e) * 64 + lane] = acc[k][t][e];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = dbacc[k][e];
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 4);
        v += __shfl_xor(v, 8);
        if (lx == 0) dbr[wave * C + 4 * g + e] = v;
      }
      __syncthreads();
      float* slab = slabs + ((long)l * PS + b) * ES;
      for (int i = tid; i < ES; i += 64 * NWAVE) {
        float v;
        if (i < 9 * C * C) {
          const int t = i >> 8, m = (i >> 4) & 15, o = i & 15;
          const int ri = ((t * 4 + (m & 3)) * 64 + (m >> 2) * 16 + o);
          v = (red[ri] + red[9 * 4 * 64 + ri]) + (red[2 * 9 * 4 * 64 + ri] + red[3 * 9 * 4 * 64 + ri]);
        } else {
          const int o = i - 9 * C * C;
          v = (dbr[o] + dbr[C + o]) + (dbr[2 * C + o] + dbr[3 * C + o]);
        }
        slab[i] = h * v;
      }
      for (int j = P + b; j < PS; j += P) {  // padding slabs of the 32-slab reduction groups
        float* zs = slabs + ((long)l * PS + j) * ES;
        for (int i = tid; i < ES; i += 64 * NWAVE) zs[i] = 0.f;
      }
      __syncthreads();
    }
    // the reduction area overlapped the x tiles: restore their zero halos
    for (int i = tid; i < 2 * TILE / 16; i += 64 * NWAVE) ((uint4*)(lds + L_X))[i] = make_uint4(0, 0, 0, 0);
    __syncthreads();
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
  const size_t lds = 2 * (size_t)deep::TILE;
  if (store_all)
    hipLaunchKernelGGL(deep::k_fwd16_fused<true>, dim3(grid), dim3(64 * deep::NWAVE), lds, s, (const bf16*)x0,
                       (bf16*)y0, y_stride, mask0, mask_stride, (const bf16*)wpack, bias, bias_stride, h, N, L);
  else
    hipLaunchKernelGGL(deep::k_fwd16_fused<false>, dim3(grid), dim3(64 * deep::NWAVE), lds, s, (const bf16*)x0,
                       (bf16*)y0, y_stride, mask0, mask_stride, (const bf16*)wpack, bias, bias_stride, h, N, L);
  ASR_LAUNCH_CHECK("k_fwd16_fused");
  return ASR_OK;
}

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
  hipLaunchKernelGGL(deep::k_bwd16_fused, dim3(P), dim3(64 * deep::NWAVE), (size_t)deep::L_TOTAL, s, (bf16*)dbufA,
                     (bf16*)dbufB, (const bf16*)xs, x_stride, masks, mask_stride, (const bf16*)wpack, h, two_gamma,
                     N, L, slabs, PS);
  ASR_LAUNCH_CHECK("k_bwd16_fused");
  *slab_rows = PS;
  *dx0_in_b = ((L + deep::KSEG - 1) / deep::KSEG) & 1;
  return ASR_OK;
}

}  // namespace asr
