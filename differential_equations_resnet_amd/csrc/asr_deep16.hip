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
      // rows software-pipelined: the B fragments of row k+1 are read during row k's MFMAs
      bf16x8 B[2][2][KS];
      auto loadB = [&](int k, bf16x8 (&Bd)[2][KS]) {
        const unsigned char* tb = src + (r0 + k) * ROWB;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          Bd[0][ks] = *(const bf16x8*)(tb + boff[ks]);
          Bd[1][ks] = *(const bf16x8*)(tb + 512 + boff[ks]);
        }
      };
      loadB(0, B[0]);
      unsigned mw[RPW][2];
#pragma unroll
      for (int k = 0; k < RPW; ++k) {
        const int r = r0 + k;
        if (k + 1 < RPW) loadB(k + 1, B[(k + 1) & 1]);
        f32x4 acc[2] = {{bz[0], bz[1], bz[2], bz[3]}, {bz[0], bz[1], bz[2], bz[3]}};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[ks], B[k & 1][0][ks], acc[0], 0, 0, 0);
          acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[ks], B[k & 1][1][ks], acc[1], 0, 0, 0);
        }
#pragma unroll
        for (int pt = 0; pt < 2; ++pt) {
          const unsigned char* tb = src + r * ROWB + pt * 512;
          // epilogue: y = x + h * relu(z) (fp32, one rounding), relu bits
          const bf16x4 xr = *(const bf16x4*)(tb + xoff);
          bf16x4 o4;
          unsigned nib = 0;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float z = acc[pt][e];
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
          mw[k][pt] = s32[0] | s32[1];
        }
      }
      // the rows' 32 mask words each (64 B per row): lanes 0-15 pixel tile 0, 16-31 tile 1
      if (ml && lane < 32) {
        const unsigned hi = lane < 16 ? 0u : ~0u;  // a select, not an index (a lane-indexed array goes to scratch)
#pragma unroll
        for (int k = 0; k < RPW; ++k)
          *(uint16_t*)(ml + ((r0 + k) * W + lane) * 2) = (uint16_t)((mw[k][0] & ~hi) | (mw[k][1] & hi));
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
// HBM only at segment boundaries.
//
// One 512-thread workgroup per CU, two waves per SIMD with split roles:
//   waves 0-3 (dgrad): image rows [8w, 8w+8): the forward's implicit GEMM on
//     dzm (bitwise the per-block kernel's dx), dx updated in place, db;
//   waves 4-6 (wgrad): tap column kx = w-4 of all 32 rows: a GEMM with M = the
//     tap's 16 input channels, N = o, K = the 32 pixels of a row.  The x
//     fragment of tile row ir (ds_read_b64_tr_b16, T10) serves the three taps
//     (ky, kx) of output rows ir - ky, so every x row is read once per wave;
//     the dz fragments of the last three rows stay in registers.  The 8
//     k-pixels of lane group g are 8g + 4*(hh ^ (g & 1)) + q for the two reads
//     hh: odd groups swap halves, so the two 16-lane groups of each 32-lane
//     half read disjoint banks;
//   wave 7 DMAs x_{l-1} and mask_{l-1} into the second buffers meanwhile.
// All 8 waves build dzm (phase 1) between two barriers.
// LDS: dx (32 KiB) | dz tile | 2 x tiles | 2 x 2 KiB masks | 4 KiB mask table.
// ---------------------------------------------------------------------------
constexpr int KSEG = 12;                 // layers per segment (dW accumulators in registers)
constexpr int NWB = 8;                   // waves per backward workgroup
constexpr int ES = 9 * C * C + C;        // slab floats per layer
constexpr int DXB = H * W * C * 2;       // 32 KiB
constexpr int MB = H * W * C / 8;        // 2 KiB of relu bits per image
constexpr int L_DX = 0, L_DZ = L_DX + DXB, L_X = L_DZ + TILE, L_M = L_X + 2 * TILE, L_TAB = L_M + 2 * MB;
constexpr int L_DBS = L_TAB + 4096;       // [KSEG][4][C] fp32 db partials
constexpr int L_TOTAL = L_DBS + KSEG * 4 * C * 4;
static_assert(L_TOTAL <= 160 * 1024, "LDS budget");

// f(integral_constant<int, k>) for k = K .. N-1: compile-time register-array
// indices (a runtime index would put the array in scratch memory)
template <int K, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (K < N) {
    f(std::integral_constant<int, K>{});
    static_for<K + 1, N>(f);
  }
}

__device__ __forceinline__ bf16x8 tr2(const unsigned char* base, const unsigned (&o)[2]) {
  return tr_pair(base + o[0], base + o[1]);
}

__global__ __launch_bounds__(64 * NWB, 1) void k_bwd16_fused(bf16* __restrict__ dbufA, bf16* __restrict__ dbufB,
                                                            const bf16* __restrict__ xs, long x_stride,
                                                            const uint8_t* __restrict__ masks, long mask_stride,
                                                            const bf16* __restrict__ wpack, float h, float two_gamma,
                                                            int N, int L, float* __restrict__ slabs, int PS) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, lx = lane & 15, q = lx >> 2, p = lx & 3;
  const int P = gridDim.x, b = blockIdx.x;
  // zero the dz tile and both x tiles (halo rows / columns stay zero), build the mask table
  for (int i = tid; i < 3 * TILE / 16; i += 64 * NWB) ((uint4*)(lds + L_DZ))[i] = make_uint4(0, 0, 0, 0);
  {
    unsigned* tab = (unsigned*)(lds + L_TAB);  // dword d of byte m: 0xffff per set bit of (m >> 2d) & 3
    for (int i = tid; i < 1024; i += 64 * NWB) {
      const unsigned m = (unsigned)i >> 2, d = (unsigned)i & 3;
      tab[i] = (((m >> (2 * d)) & 1u) ? 0xffffu : 0u) | (((m >> (2 * d + 1)) & 1u) ? 0xffff0000u : 0u);
    }
  }
  __syncthreads();
  const int nseg = (L + KSEG - 1) / KSEG;
  const int wv = __builtin_amdgcn_readfirstlane(wave);

  // ---- role-independent steps (every wave takes part; identical barrier sequence) ----
  // dx at the segment top, x_ltop and mask_ltop of image n: 66 DMAs dealt round-robin
  auto stage = [&](const bf16* din, long img, int ltop, int n) {
    const unsigned char* ds = (const unsigned char*)(din + img);
    const unsigned char* xsrc = (const unsigned char*)(xs + ltop * x_stride + img);
    for (int j = wv; j < 66; j += NWB) {
      if (j < 32) dma16(ds + j * 1024 + lane * 16, lds + L_DX + j * 1024);
      else if (j < 64) dma16(xsrc + (j - 32) * 1024 + lane * 16, lds + L_X + (j - 31) * ROWB + 32);
      else dma16(masks + ltop * mask_stride + (long)n * MB + (j - 64) * 1024 + lane * 16, lds + L_M + (j - 64) * 1024);
    }
  };
  // phase 1: dzm = dx & mask (cur mask buffer) for the whole image, 4 chunks per thread
  // (all reads first, so their latencies overlap)
  auto build_dz = [&](int cur) {
    const unsigned char* mt = lds + L_M + cur * MB;
    uint4 dv[4], mv[4];
    unsigned mb[4], zo[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = tid + 64 * NWB * j;
      const int r = c >> 6, px = (c & 63) >> 1, hc = c & 1;
      dv[j] = *(const uint4*)(lds + L_DX + (r * W + px) * 32 + hc * 16);
      mb[j] = mt[(r * W + px) * 2 + hc];
      zo[j] = (unsigned)(((r + 1) * TW + px + 1) * 32 + hc * 16);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) mv[j] = *(const uint4*)(lds + L_TAB + mb[j] * 16);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      *(uint4*)(lds + L_DZ + zo[j]) = make_uint4(dv[j].x & mv[j].x, dv[j].y & mv[j].y, dv[j].z & mv[j].z,
                                                 dv[j].w & mv[j].w);
  };
  auto store_dx = [&](bf16* dout, long img) {
    unsigned char* dst = (unsigned char*)(dout + img);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int o = (tid + j * 64 * NWB) * 16;
      *(uint4*)(dst + o) = *(const uint4*)(lds + L_DX + o);
    }
  };
  float* dbs = (float*)(lds + L_DBS);  // [KSEG][4 dgrad waves][C] db partial sums of the segment

  if (wave < 4) {
    // ------------------------------ dgrad waves ------------------------------
    const int r0 = wave * RPW;
    const float hs2g = h * two_gamma;
    unsigned boff[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int tap = min(2 * ks + (g >> 1), 8);
      boff[ks] = (unsigned)(((tap / 3) * TW + tap % 3 + lx) * 32 + (g & 1) * 16);
    }
    const unsigned zoff = (unsigned)((TW + 1 + lx) * 32 + 8 * g);  // dz interior value of the D layout
    const unsigned doff = (unsigned)(lx * 32 + 8 * g);              // dx (no halo) of the D layout
    for (int sg = 0; sg < nseg; ++sg) {
      const int ltop = L - 1 - sg * KSEG, kcount = min(KSEG, ltop + 1);
      const bf16* din = (sg & 1) ? dbufB : dbufA;
      bf16* dout = (sg & 1) ? dbufA : dbufB;
      for (int i = lane; i < KSEG * C; i += 64) dbs[(i / C) * 4 * C + wave * C + i % C] = 0.f;
      for (int n = b; n < N; n += P) {
        const long img = (long)n * H * W * C;
        stage(din, img, ltop, n);
        bf16x8 A[KS], An[KS];
        load_wt(wpack + (long)ltop * WSTRIDE, lane, A);
        barrier_vm(0);
        for (int k = 0; k < kcount; ++k) {
          const int l = ltop - k;
          const bool more = k + 1 < kcount;
          if (more) load_wt(wpack + (long)(l - 1) * WSTRIDE, lane, An);
          build_dz(k & 1);
          barrier_lds();  // dzm complete (the prefetch DMA keeps flying)
          float dsum[4] = {0.f, 0.f, 0.f, 0.f};
          // rows software-pipelined: the B fragments of row j+1 are read during row j's MFMAs
          bf16x8 B[2][2][KS];
          auto loadB = [&](int j, bf16x8 (&Bd)[2][KS]) {
            const unsigned char* tb = lds + L_DZ + (r0 + j) * ROWB;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
              Bd[0][ks] = *(const bf16x8*)(tb + boff[ks]);
              Bd[1][ks] = *(const bf16x8*)(tb + 512 + boff[ks]);
            }
          };
          loadB(0, B[0]);
#pragma unroll
          for (int j = 0; j < RPW; ++j) {
            const int r = r0 + j;
            if (j + 1 < RPW) loadB(j + 1, B[(j + 1) & 1]);
            f32x4 c[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
              c[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[ks], B[j & 1][0][ks], c[0], 0, 0, 0);
              c[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[ks], B[j & 1][1][ks], c[1], 0, 0, 0);
            }
            const unsigned char* tb = lds + L_DZ + r * ROWB;
#pragma unroll
            for (int pt = 0; pt < 2; ++pt) {
              const bf16x4 zr = *(const bf16x4*)(tb + pt * 512 + zoff);
              unsigned char* dxp = lds + L_DX + (r * W + 16 * pt) * 32 + doff;
              const bf16x4 dr = *(const bf16x4*)dxp;
              bf16x4 o4;
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const float zf = (float)zr[e];
                dsum[e] += zf;
                const float v = fmaf(-h, c[pt][e], (float)dr[e]);
                o4[e] = (bf16)(hs2g != 0.f ? fmaf(hs2g, zf, v) : v);
              }
              *(bf16x4*)dxp = o4;
            }
          }
          // db of this layer: the wave's 16 pixel lanes, added to its own slot (no other writer)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float v = dsum[e];
            v += __shfl_xor(v, 1);
            v += __shfl_xor(v, 2);
            v += __shfl_xor(v, 4);
            v += __shfl_xor(v, 8);
            if (lx == 0) dbs[(k * 4 + wave) * C + 4 * g + e] += v;
          }
          if (more) {
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) A[ks] = An[ks];
          }
          barrier_vm(0);  // dx updated, dz and x_l consumed; x_{l-1} / mask_{l-1} landed
        }
        store_dx(dout, img);
        barrier_lds();  // dx read out before the next image's DMA overwrites it
      }
      // segment end: db of each layer, the four dgrad waves summed in a fixed order
      __syncthreads();
      if (tid < C)
        for (int k = 0; k < kcount; ++k) {
          const float* d = dbs + k * 4 * C + tid;
          slabs[((long)(ltop - k) * PS + b) * ES + 9 * C * C + tid] = h * ((d[0] + d[C]) + (d[2 * C] + d[3 * C]));
        }
      __syncthreads();
    }
  } else {
    // ------------------------------ wgrad waves ------------------------------
    const int kx = wave - 4;  // 0..2; wave 7: prefetch only
    unsigned to2[2];          // tr-read lane offsets (pixel 8g + 4*(hh ^ (g&1)) + q, channels 4p..4p+3)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) to2[hh] = (unsigned)((8 * g + 4 * (hh ^ (g & 1)) + q) * 32 + 8 * p);
    f32x4 acc[KSEG][3];
    // one layer's weight gradient for tap column kx into a[ky] (ky = 0..2): x fragment of
    // tile row ir feeds output rows ir - ky; reads run DEPTH rows ahead of the MFMAs
    auto wgrad_layer = [&](f32x4 (&a)[3], int cur) {
      constexpr int DEPTH = 2;
      const unsigned char* xt = lds + L_X + cur * TILE + kx * 32;  // tile column pixel + kx
      const unsigned char* zt = lds + L_DZ + ROWB + 32;           // dz of output row 0, pixel 0
      bf16x8 Aq[DEPTH + 1], Bq[DEPTH + 1];
      const bf16x8 Bz = tr2(zt, to2);  // B of output row 0
#pragma unroll
      for (int d = 1; d <= DEPTH; ++d) {
        Aq[d % (DEPTH + 1)] = tr2(xt + d * ROWB, to2);
        if (d < H) Bq[d % (DEPTH + 1)] = tr2(zt + d * ROWB, to2);
      }
      bf16x8 Bm1 = Bz, Bm2 = Bz;
#pragma unroll
      for (int ir = 1; ir <= H; ++ir) {  // tile rows holding image rows 0 .. 31
        if (ir + DEPTH <= H) {
          Aq[(ir + DEPTH) % (DEPTH + 1)] = tr2(xt + (ir + DEPTH) * ROWB, to2);
          if (ir + DEPTH < H) Bq[(ir + DEPTH) % (DEPTH + 1)] = tr2(zt + (ir + DEPTH) * ROWB, to2);
        }
        const bf16x8 Ax = Aq[ir % (DEPTH + 1)];
        if (ir < H) a[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ax, Bq[ir % (DEPTH + 1)], a[0], 0, 0, 0);  // ky=0
        a[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ax, Bm1, a[1], 0, 0, 0);  // ky=1: output row ir-1
        if (ir >= 2) a[2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ax, Bm2, a[2], 0, 0, 0);  // ky=2: row ir-2
        Bm2 = Bm1;
        if (ir < H) Bm1 = Bq[ir % (DEPTH + 1)];
      }
    };
    for (int sg = 0; sg < nseg; ++sg) {
      const int ltop = L - 1 - sg * KSEG, kcount = min(KSEG, ltop + 1);
      const bf16* din = (sg & 1) ? dbufB : dbufA;
#pragma unroll
      for (int k = 0; k < KSEG; ++k)
#pragma unroll
        for (int t = 0; t < 3; ++t) acc[k][t] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int n = b; n < N; n += P) {
        const long img = (long)n * H * W * C;
        stage(din, img, ltop, n);
        barrier_vm(0);
        for (int k = 0; k < kcount; ++k) {
          const int l = ltop - k, cur = k & 1;
          if (wave == 7 && k + 1 < kcount) {  // x_{l-1}, mask_{l-1} into the other buffers
            const unsigned char* xsrc = (const unsigned char*)(xs + (l - 1) * x_stride + img);
            for (int j = 0; j < 32; ++j)
              dma16(xsrc + j * 1024 + lane * 16, lds + L_X + (cur ^ 1) * TILE + (j + 1) * ROWB + 32);
            for (int j = 0; j < 2; ++j)
              dma16(masks + (l - 1) * mask_stride + (long)n * MB + j * 1024 + lane * 16,
                    lds + L_M + (cur ^ 1) * MB + j * 1024);
          }
          build_dz(cur);
          barrier_lds();
          if (wave < 7) {  // this layer's accumulators (a compile-time index per branch)
            static_for<0, KSEG>([&](auto kc) {
              if (k == decltype(kc)::value) wgrad_layer(acc[decltype(kc)::value], cur);
            });
          }
          barrier_vm(0);
        }
        store_dx((sg & 1) ? dbufA : dbufB, img);
        barrier_lds();
      }
      // segment end: dW of each layer straight from the accumulators (complete sums)
      __syncthreads();
      static_for<0, KSEG>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        if (k >= kcount) return;
        float* slab = slabs + ((long)(ltop - k) * PS + b) * ES;
        if (wave < 7) {
#pragma unroll
          for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int e = 0; e < 4; ++e) slab[((3 * ky + kx) * 16 + 4 * g + e) * 16 + lx] = h * acc[k][ky][e];
        } else {
          for (int j = P + b; j < PS; j += P) {  // padding slabs of the 32-slab reduction groups
            float* zs = slabs + ((long)(ltop - k) * PS + j) * ES;
            for (int i = lane; i < ES; i += 64) zs[i] = 0.f;
          }
        }
      });
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
  hipLaunchKernelGGL(deep::k_bwd16_fused, dim3(P), dim3(64 * deep::NWB), (size_t)deep::L_TOTAL, s, (bf16*)dbufA,
                     (bf16*)dbufB, (const bf16*)xs, x_stride, masks, mask_stride, (const bf16*)wpack, h, two_gamma,
                     N, L, slabs, PS);
  ASR_LAUNCH_CHECK("k_bwd16_fused");
  *slab_rows = PS;
  *dx0_in_b = ((L + deep::KSEG - 1) / deep::KSEG) & 1;
  return ASR_OK;
}

}  // namespace asr
