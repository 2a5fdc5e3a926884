// fp32 path of the 3x3 conv / Euler block: fp32 MFMA (v_mfma_f32_16x16x4_f32)
// for the network's blocks (C in {16, 32, 64}, W in {32, 16, 8}: the single-stage
// nets and the stages of the multi-stage ones), exact fp32 FMA chains on the
// VALU for every other shape.
//
// This is the reference-precision path (the reference computes everything in
// fp32, layers/tfkeras_layer_Conv2DAntisymmetric3By3.py:157-171), used for the
// fp32 parity configuration (BASELINE config 1), for shapes the bf16 MFMA
// kernels do not cover, and for the stem conv (models/tfkeras_resnets.py:563-572,
// a regular 3x3 conv with C_in = 3).  It shares the mask layout, the theta
// projection and the API with the bf16 path.
#include "asr_common.h"

namespace asr {

enum { F_EULER = 0, F_CONV = 1, F_RELU = 2, B_EULER = 3, B_CONV = 4 };

// One wave = (n, y, 16-pixel tile, 16-channel tile).  Lane (g = lane>>4,
// lx = lane&15) computes pixel 16*pt+lx, channels 16*ot+4g .. +3 (the MFMA D
// fragment map).  Relu mask: bit (pixel*C + o) (asr.h), set with atomicOr on
// a zeroed buffer because C need not be a multiple of 8 here.  K x K kernel
// (odd K, SAME: pad K/2), HWIO weights [K][K][Ci][Co].
template <typename Tin, typename Tout, int MODE>
__global__ __launch_bounds__(256) void k_conv_f32(const Tin* __restrict__ xin, Tout* __restrict__ out,
                                                  uint32_t* __restrict__ mask, const float* __restrict__ w,
                                                  const float* __restrict__ bias, float h, float two_gamma,
                                                  const float* __restrict__ dy, const float* __restrict__ extra,
                                                  int N, int H, int W, int Ci, int Co, int K) {
  const int PT = (W + 15) / 16, OT = (Co + 15) / 16;
  const long tasks = (long)N * H * PT * OT;
  const long task = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (task >= tasks) return;
  const int lane = threadIdx.x & 63, g = lane >> 4, lx = lane & 15;
  const int ot = (int)(task % OT);
  long rest = task / OT;
  const int pt = (int)(rest % PT);
  rest /= PT;
  const int y = (int)(rest % H);
  const int n = (int)(rest / H);
  const int px = 16 * pt + lx;
  const int o0 = 16 * ot + 4 * g;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  if (px < W) {
    for (int tap = 0; tap < K * K; ++tap) {
      const int gy = y + tap / K - K / 2, gx = px + tap % K - K / 2;
      if (gy < 0 || gy >= H || gx < 0 || gx >= W) continue;
      const Tin* xp = xin + (((long)n * H + gy) * W + gx) * Ci;
      const float* wp = w + (long)tap * Ci * Co;
      for (int i = 0; i < Ci; ++i) {
        const float xv = to_f32(xp[i]);
        const float* wr = wp + (long)i * Co + o0;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (o0 + e < Co) acc[e] = fmaf(xv, wr[e], acc[e]);
      }
    }
  }
  const long pix = (((long)n * H + y) * W + px);
  unsigned nib = 0;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int o = o0 + e;
    const bool ok = px < W && o < Co;
    float v = 0.f;
    if constexpr (MODE <= F_RELU) {
      const float z = acc[e] + ((bias && o < Co) ? bias[o] : 0.f);
      if constexpr (MODE == F_EULER) {
        if (ok && z > 0.f) nib |= 1u << e;
        // residual: the input, or `extra` (the step input of the second RK2 stage)
        if (ok) v = (extra ? extra[pix * Co + o] : to_f32(xin[pix * Ci + o])) + h * fmaxf(z, 0.f);
      } else if constexpr (MODE == F_CONV) {
        v = z;
      } else {
        v = fmaxf(z, 0.f);
      }
    } else {
      // dgrad: xin holds dz (float), dy the incoming gradient (float)
      if (ok) {
        const float dz = to_f32(xin[pix * Ci + o]);
        v = (MODE == B_EULER ? dy[pix * Co + o] : 0.f) - acc[e] + two_gamma * dz;
        if (extra) v += extra[pix * Co + o];  // RK2 first stage: + the step's outer dy
      }
    }
    if (ok) out[pix * Co + o] = from_f32<Tout>(v);
  }
  if constexpr (MODE == F_EULER) {
    if (mask && nib) {
      const long b0 = pix * Co + o0;  // first of this lane's 4 channels
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if ((nib >> e) & 1u) atomicOr(mask + ((b0 + e) >> 5), 1u << ((b0 + e) & 31));
    }
  }
}

// dz = h*dy*mask (EULER), dy (CONV) or dy*[src > 0] (RELU), as float.
template <typename T>
__global__ void k_make_dz(const T* __restrict__ dy, const uint8_t* __restrict__ mask, const T* __restrict__ relu_src,
                          int mode, float h, int N, int H, int W, int C, float* __restrict__ dz) {
  const long P = (long)N * H * W * C;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < P; idx += (long)gridDim.x * blockDim.x) {
    const float d = to_f32(dy[idx]);
    float v = d;
    if (mode == F_EULER) {
      v = ((mask[idx >> 3] >> (idx & 7)) & 1) ? h * d : 0.f;  // bit idx = pixel*C + o
    } else if (mode == F_RELU) {
      v = to_f32(relu_src[idx]) > 0.f ? d : 0.f;
    }
    dz[idx] = v;
  }
}

// dW[tap][i][o] partial over a chunk of image rows:
//   slab[chunk][(tap*Ci + i)*Co + o] = sum_{rows in chunk, px} x[p+s(tap)][i] * dz[p][o]
// (slab rows are E + Co floats: dW partial then the db partial of k_db_f32)
template <typename Tx>
__global__ __launch_bounds__(256) void k_wgrad_f32(const Tx* __restrict__ x, const float* __restrict__ dz, int N,
                                                   int H, int W, int Ci, int Co, int rows_per_chunk,
                                                   float* __restrict__ slabs, int K) {
  const long E = (long)K * K * Ci * Co;
  const long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (e >= E) return;
  const int o = (int)(e % Co);
  const int i = (int)((e / Co) % Ci);
  const int tap = (int)(e / ((long)Ci * Co));
  const int sy = tap / K - K / 2, sx = tap % K - K / 2;
  const long R = (long)N * H;
  const long r0 = (long)blockIdx.y * rows_per_chunk, r1 = min(R, r0 + rows_per_chunk);
  float acc = 0.f;
  for (long rr = r0; rr < r1; ++rr) {
    const int y = (int)(rr % H);
    const int n = (int)(rr / H);
    const int gy = y + sy;
    if (gy < 0 || gy >= H) continue;
    const Tx* xr = x + ((long)n * H + gy) * W * Ci;
    const float* dr = dz + ((long)n * H + y) * W * Co;
    const int p0 = max(0, -sx), p1 = min(W, W - sx);
    for (int p = p0; p < p1; ++p) acc = fmaf(to_f32(xr[(long)(p + sx) * Ci + i]), dr[(long)p * Co + o], acc);
  }
  slabs[(long)blockIdx.y * (E + Co) + e] = acc;
}

// db partial per chunk of pixel rows, into the slab row tail: slabs[chunk][E + o]
__global__ void k_db_f32(const float* __restrict__ dz, long rows, int W, int C, int rows_per_chunk, long E,
                         float* __restrict__ slabs) {
  const int o = threadIdx.x;
  if (o >= C) return;
  const long r0 = (long)blockIdx.x * rows_per_chunk, r1 = min(rows, r0 + rows_per_chunk);
  float acc = 0.f;
  for (long p = r0 * W; p < r1 * W; ++p) acc += dz[p * C + o];
  slabs[(long)blockIdx.x * (E + C) + E + o] = acc;
}

// ===========================================================================
// fp32 on the matrix cores: v_mfma_f32_16x16x4_f32 (fp32 operands, fp32
// accumulation: the reference's precision, …3By3.py:157-171) for the 3x3
// SAME conv / Euler block with C_in = C_out = C in {16, 32, 64}, W in {32, 16, 8}.
//
// Forward / dgrad (k_conv32): implicit GEMM D[o][px] = sum_kappa W^T[o][kappa]
// X[kappa][px], kappa = (tap, i).  A workgroup (4 waves) owns a band of BR = 4
// output rows of one image: the BR + 2 input rows (zero rows outside the
// image, zero halo columns) are staged in LDS once, every wave keeps its
// o-tile's A = W^T fragments in registers for the launch (9C/4 VGPRs) and
// walks its share of the band's 16-pixel tiles (band pixel 16 tile + lx; at
// W = 8 a tile spans two rows; C=16: the 4 waves deal the tiles round-robin;
// C=64: one o-tile per wave, every tile).  K-step s of channel group q at a tap gives lane (lx, g) the
// channel 16q + 4g + s, so one 16-B LDS read per lane (the pixel's channels
// 16q+4g .. +3) feeds four MFMAs.  The accumulator lane (lx, g) holds
// channels 4g .. 4g+3 of pixel lx: the residual / dy / dz operands and the
// output are 16-B accesses, and the relu-mask nibbles of a pixel's 16
// channels are merged across the 4 lane groups into one 16-bit store (every
// bit written: no memset, no atomics).
// Weight gradient (k_wgrad32): D[i][o] = sum_px x[px + tap][i] dz[px][o] per
// tap, K = 4 pixels per MFMA (one fp32 per lane from LDS for each operand).
// 12 waves: (tap row ky, o-tile, row split); each holds the 3 taps of its row
// x C/16 i-tiles of its o-tile in accumulators over a persistent run of
// bands, the row-split partials are summed through LDS at the end and the
// workgroup writes one [dW | db] slab (db on MFMA: ones x dz in the ky = 1
// waves), reduced by the same two-pass k_reduce_slabs / projection as the
// bf16 path.
// ===========================================================================
template <int C, int W_>
struct F32Band {
  // pixel strides in LDS (floats), padded against bank conflicts: PSC for the conv's 16-B reads
  // (16 lanes = 16 consecutive pixels on distinct banks), PSW for the wgrad's 4-B reads (the two
  // lane groups of a 32-lane half, one pixel apart, on disjoint banks); unpadded, a C = 64 tile
  // put the 16 lanes of a conv read on one bank group
  static constexpr int PSC = C + 4, PSW = C >= 32 ? C + 16 : C;
  static constexpr int OT = C / 16, W = W_, TW = W + 2, BR = 4, TILEF = (BR + 2) * TW * PSC;
  static constexpr int TILEW = (BR + 2) * TW * PSW;  // the wgrad's x tile
  static constexpr int T = BR * W / 16;  // 16-pixel tiles per band (band pixel p = 16 tile + lx: row p / W, col p % W)
  static constexpr int WPT = 4 / OT;    // forward / dgrad: waves sharing an o-tile, tiles dealt round-robin
  static constexpr int RS = 4 / OT;     // wgrad row split: 3 * OT * RS = 12 waves
  static constexpr int DZF = BR * W * PSW;
  static_assert(W == 8 || W == 16 || W == 32, "fp32 MFMA band: W in {8, 16, 32}");
};

// 4 consecutive elements as fp32 (a 16-B load, or 8 B of bf16 converted)
__device__ __forceinline__ f32x4 load4f(const float* p) { return *(const f32x4*)p; }
__device__ __forceinline__ f32x4 load4f(const bf16* p) {
  const uint2 u = *(const uint2*)p;
  return f32x4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
               __uint_as_float(u.y & 0xffff0000u)};
}

// dz = h dy [relu bit] of 4 channels (bit index pixel*C + c, C a multiple of 16: a nibble)
__device__ __forceinline__ f32x4 masked_dz4(f32x4 v, const uint8_t* __restrict__ dmask, long bit, float dh) {
  const unsigned nib = (unsigned)(dmask[bit >> 3] >> (bit & 7));
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = ((nib >> j) & 1u) ? dh * v[j] : 0.f;
  return v;
}

// stage rows y0-1 .. y0+BR of image n into tile (zeros outside the image and
// in the two halo columns), float4 per thread; with dmask, src is dy and the
// tile gets dz = dh * dy * [relu bit] (the Euler block's dz, no separate pass)
template <int C, int W, typename Ts = float, int PS = C, int NT = 256>
__device__ __forceinline__ void f32_stage_rows(const Ts* __restrict__ src, float* tile, int n, int y0, int H,
                                               int tid, const uint8_t* __restrict__ dmask = nullptr,
                                               float dh = 1.f) {
  using G = F32Band<C, W>;
  constexpr int C4 = C / 4, NCH = (G::BR + 2) * G::TW * C4, NIT = (NCH + NT - 1) / NT, B = 4;
  // B loads in flight before their stores (a rolled loop waited for each load in turn)
#pragma unroll
  for (int k0 = 0; k0 < NIT; k0 += B) {
    f32x4 v[B];
    long ev[B];
    unsigned mb[B];  // the relu byte of each element (with dmask), loaded beside its values
#pragma unroll
    for (int k = 0; k < B; ++k) {
      const int i = tid + (k0 + k) * NT;
      const int r = i / (G::TW * C4), rem = i % (G::TW * C4), col = rem / C4, c4 = rem % C4;
      const int gy = y0 - 1 + r, gx = col - 1;
      v[k] = f32x4{0.f, 0.f, 0.f, 0.f};
      ev[k] = -1;
      mb[k] = 0u;
      if (k0 + k < NIT && i < NCH && (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)G::W) {
        ev[k] = (((long)n * H + gy) * G::W + gx) * C + 4 * c4;
        v[k] = load4f(src + ev[k]);
        if (dmask) mb[k] = dmask[ev[k] >> 3];
      }
    }
#pragma unroll
    for (int k = 0; k < B; ++k) {
      const int i = tid + (k0 + k) * NT;
      if (k0 + k < NIT && i < NCH) {
        const int r = i / (G::TW * C4), rem = i % (G::TW * C4), col = rem / C4, c4 = rem % C4;
        if (dmask && ev[k] >= 0) {  // (masked_dz4 on the preloaded byte: dz = dh dy [relu bit])
          const unsigned nib = mb[k] >> (ev[k] & 7);
#pragma unroll
          for (int j = 0; j < 4; ++j) v[k][j] = ((nib >> j) & 1u) ? dh * v[k][j] : 0.f;
        }
        *(f32x4*)(tile + (r * G::TW + col) * PS + 4 * c4) = v[k];
      }
    }
  }
}

template <int C, int W, int MODE>
__global__ __launch_bounds__(256) void k_conv32(const float* __restrict__ xin, float* __restrict__ out,
                                                uint8_t* __restrict__ mask, const float* __restrict__ w,
                                                const float* __restrict__ bias, float h, float two_gamma,
                                                const float* __restrict__ dy, const float* __restrict__ extra, int N,
                                                int H, const uint8_t* __restrict__ dmask) {
  using G = F32Band<C, W>;
  constexpr int OT = G::OT, TW = G::TW, BR = G::BR;
  __shared__ __attribute__((aligned(16))) float tile[G::TILEF];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, lx = lane & 15;
  const int ot = wave % OT, rw = wave / OT;
  const int nb = (H + BR - 1) / BR;
  const int n = blockIdx.x / nb, y0 = (blockIdx.x % nb) * BR;
  if (n >= N) return;
  // A = W^T of o-tile ot (HWIO W): A[t][q][s] = W[t][16q + 4g + s][16 ot + lx]
  float A[9][OT][4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int q = 0; q < OT; ++q)
#pragma unroll
      for (int s = 0; s < 4; ++s) A[t][q][s] = w[((long)t * C + 16 * q + 4 * g + s) * C + 16 * ot + lx];
  f32x4 bz = {0.f, 0.f, 0.f, 0.f};
  if (MODE <= F_RELU && bias) bz = *(const f32x4*)(bias + 16 * ot + 4 * g);
  // (backward with dmask: xin is dy, the tile gets dz = h dy [relu bit])
  f32_stage_rows<C, W, float, G::PSC, 256>(xin, tile, n, y0, H, tid, MODE >= B_EULER ? dmask : nullptr, h);
  __syncthreads();
  // wave (ot, rw) takes the band's 16-pixel tiles rw, rw + WPT, ..; lane lx's pixel of tile tau is band
  // pixel 16 tau + lx (W = 8: a tile spans two rows, so validity is per lane)
  constexpr int NT = (G::T + G::WPT - 1) / G::WPT;
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int tau = rw + j * G::WPT;
    if (tau >= G::T) break;  // (wave-uniform)
    const int bp = 16 * tau + lx, r = bp / W, px = bp % W;
    if (W >= 16 && y0 + r >= H) break;  // (wave-uniform for W >= 16; rows only grow with tau)
    f32x4 acc = bz;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int q = 0; q < OT; ++q) {
        const f32x4 bv = *(const f32x4*)(tile + ((r + t / 3) * TW + px + t % 3) * G::PSC + 16 * q + 4 * g);
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A[t][q][s], bv[s], acc, 0, 0, 0);
      }
    mfma_f32_settle();  // (the epilogue branches: every path must see the result's wait states)
    {
      const bool ok = y0 + r < H;
      const long pix = ((long)n * H + y0 + r) * W + px;
      const long oi = pix * C + 16 * ot + 4 * g;  // this lane's 4 channels
      const f32x4 ctr = *(const f32x4*)(tile + ((r + 1) * TW + px + 1) * G::PSC + 16 * ot + 4 * g);  // x or dz at the pixel
      f32x4 v;
      if constexpr (MODE == F_EULER) {
        const f32x4 res = (extra && ok) ? *(const f32x4*)(extra + oi) : ctr;
        unsigned nib = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float z = acc[e];
          nib |= (z > 0.f ? 1u : 0u) << e;
          v[e] = res[e] + h * fmaxf(z, 0.f);
        }
        if (mask) {  // the pixel's 16 channels of this o-tile: 4 nibbles, one 16-bit store
          unsigned m = nib << (4 * g);
          m |= (unsigned)__shfl_xor((int)m, 16, 64);
          m |= (unsigned)__shfl_xor((int)m, 32, 64);
          if (g == 0 && ok) *(uint16_t*)(mask + (pix * C + 16 * ot) / 8) = (uint16_t)m;
        }
      } else if constexpr (MODE == F_CONV) {
        v = acc;
      } else {  // B_EULER / B_CONV: the tile holds dz; dx = [dy] - A dz + 2 gamma dz [+ extra]
        f32x4 d0 = {0.f, 0.f, 0.f, 0.f};
        if (ok) {
          if constexpr (MODE == B_EULER) d0 = *(const f32x4*)(dy + oi);
          if (extra) d0 += *(const f32x4*)(extra + oi);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = d0[e] - acc[e] + two_gamma * ctr[e];
      }
      if (ok) *(f32x4*)(out + oi) = v;
    }
  }
}

template <int C, int W, typename Tx = float>
__global__ __launch_bounds__(768) void k_wgrad32(const Tx* __restrict__ x, const Tx* __restrict__ dz, int N,
                                                 int H, float* __restrict__ slabs, const uint8_t* __restrict__ dmask,
                                                 float dh, long x_stride = 0, long dz_stride = 0, long m_stride = 0,
                                                 long s_stride = 0) {
  using G = F32Band<C, W>;
  // several layers in one launch: blockIdx.y is the layer
  x += blockIdx.y * x_stride;
  dz += blockIdx.y * dz_stride;
  if (dmask) dmask += blockIdx.y * m_stride;
  slabs += blockIdx.y * s_stride;
  constexpr int OT = G::OT, TW = G::TW, BR = G::BR, RS = G::RS, E = 9 * C * C;
  extern __shared__ __attribute__((aligned(16))) float lds32[];
  float* xt = lds32;               // [BR+2][TW][C]
  float* dzt = lds32 + G::TILEW;   // [BR][W][PSW]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, lx = lane & 15;
  const int ky = wave / (OT * RS), ot = (wave / RS) % OT, rs = wave % RS;
  const int nb = (H + BR - 1) / BR;
  const long items = (long)N * nb;
  const long i0 = (long)blockIdx.x * items / gridDim.x, i1 = (long)(blockIdx.x + 1) * items / gridDim.x;
  f32x4 acc[3][OT], accb = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kx = 0; kx < 3; ++kx)
#pragma unroll
    for (int it = 0; it < OT; ++it) acc[kx][it] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (long item = i0; item < i1; ++item) {
    const int n = (int)(item / nb), y0 = (int)(item % nb) * BR;
    const int rows = min(BR, H - y0);
    __syncthreads();  // the previous item's tiles consumed
    f32_stage_rows<C, W, Tx, G::PSW, 768>(x, xt, n, y0, H, tid);
    for (int i = tid; i < BR * G::W * C / 4; i += 768) {
      const int r = i / (G::W * C / 4);
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (r < rows) {
        const long e = ((long)n * H + y0) * G::W * C + 4 * i;
        v = load4f(dz + e);
        if (dmask) v = masked_dz4(v, dmask, e, dh);  // dz is dy here: dz = dh dy [relu bit]
      }
      *(f32x4*)(dzt + (i / (C / 4)) * G::PSW + 4 * (i % (C / 4))) = v;
    }
    __syncthreads();
    for (int r = rs; r < rows; r += RS) {
#pragma unroll
      for (int s = 0; s < G::W / 4; ++s) {
        const int p = 4 * s + g;  // this lane's pixel (k index) of the step
        const float bv = dzt[(r * G::W + p) * G::PSW + 16 * ot + lx];
#pragma unroll
        for (int kx = 0; kx < 3; ++kx)
#pragma unroll
          for (int it = 0; it < OT; ++it) {
            const float av = xt[((r + ky) * TW + p + kx) * G::PSW + 16 * it + lx];
            acc[kx][it] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[kx][it], 0, 0, 0);
          }
        if (ky == 1) accb = __builtin_amdgcn_mfma_f32_16x16x4f32(1.f, bv, accb, 0, 0, 0);
      }
    }
  }
  // sum the RS row-split partials through LDS (fixed order), one slab per workgroup
  constexpr int PW = (3 * OT + 1) * 256;  // floats per wave: its tiles, then db
  if constexpr (RS > 1) {
    __syncthreads();  // (the last item's tiles consumed)
    if (rs != 0) {
      float* mine = lds32 + wave * PW;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx)
#pragma unroll
        for (int it = 0; it < OT; ++it) *(f32x4*)(mine + ((kx * OT + it) * 64 + lane) * 4) = acc[kx][it];
      *(f32x4*)(mine + (3 * OT * 64 + lane) * 4) = accb;
    }
    __syncthreads();
    if (rs == 0) {
#pragma unroll
      for (int q = 1; q < RS; ++q) {
        const float* th = lds32 + (wave + q) * PW;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx)
#pragma unroll
          for (int it = 0; it < OT; ++it) acc[kx][it] += *(const f32x4*)(th + ((kx * OT + it) * 64 + lane) * 4);
        accb += *(const f32x4*)(th + (3 * OT * 64 + lane) * 4);
      }
    }
  }
  if (rs == 0) {
    float* slab = slabs + (long)blockIdx.x * (E + C);
#pragma unroll
    for (int kx = 0; kx < 3; ++kx)
#pragma unroll
      for (int it = 0; it < OT; ++it)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          slab[((long)(3 * ky + kx) * C + 16 * it + 4 * g + j) * C + 16 * ot + lx] = acc[kx][it][j];
    // db: the ky = 1 waves' ones x dz (every row of that product is the column sum)
    if (ky == 1 && g == 0) slab[E + 16 * ot + lx] = accb[0];
  }
}

template <int C, int W>
static size_t wgrad32_lds() {
  using G = F32Band<C, W>;
  const size_t stage = (size_t)(G::TILEW + G::DZF) * 4;
  const size_t red = G::RS > 1 ? (size_t)12 * (3 * G::OT + 1) * 256 * 4 : 0;
  return std::max(stage, red);
}

// the multi-stage nets' 16x16 and 8x8 stages (asr_stages.hip) run the same kernels at W = 16 / 8
static bool conv32_supported(int W, int Ci, int Co) {
  return (W == 32 || W == 16 || W == 8) && Ci == Co && (Ci == 16 || Ci == 32 || Ci == 64);
}

template <int C, int W, int MODE>
static int launch_conv32(const void* xin, void* out, uint8_t* mask, const float* w, const float* bias, float h,
                         float two_gamma, const float* dy, const float* extra, int N, int H, hipStream_t s,
                         const uint8_t* dmask = nullptr) {
  const long blocks = (long)N * ((H + 3) / 4);
  if (blocks > 0x7fffffffL) return fail(ASR_E_ARG, "conv f32: problem too large");
  hipLaunchKernelGGL((k_conv32<C, W, MODE>), dim3((unsigned)blocks), dim3(256), 0, s, (const float*)xin,
                     (float*)out, mask, w, bias, h, two_gamma, dy, extra, N, H, dmask);
  ASR_LAUNCH_CHECK("k_conv32");
  return ASR_OK;
}

template <int C, int MODE>
static int conv32_dispatch_w(int W, const void* xin, void* out, uint8_t* mask, const float* w, const float* bias,
                             float h, float two_gamma, const float* dy, const float* extra, int N, int H,
                             hipStream_t s, const uint8_t* dmask) {
  switch (W) {
    case 32: return launch_conv32<C, 32, MODE>(xin, out, mask, w, bias, h, two_gamma, dy, extra, N, H, s, dmask);
    case 16: return launch_conv32<C, 16, MODE>(xin, out, mask, w, bias, h, two_gamma, dy, extra, N, H, s, dmask);
    case 8: return launch_conv32<C, 8, MODE>(xin, out, mask, w, bias, h, two_gamma, dy, extra, N, H, s, dmask);
  }
  return fail(ASR_E_UNSUPPORTED, "conv f32 (MFMA): W=%d", W);
}

template <int MODE>
static int conv32_dispatch(int C, int W, const void* xin, void* out, uint8_t* mask, const float* w, const float* bias,
                           float h, float two_gamma, const float* dy, const float* extra, int N, int H, hipStream_t s,
                           const uint8_t* dmask = nullptr) {
  switch (C) {
    case 16: return conv32_dispatch_w<16, MODE>(W, xin, out, mask, w, bias, h, two_gamma, dy, extra, N, H, s, dmask);
    case 32: return conv32_dispatch_w<32, MODE>(W, xin, out, mask, w, bias, h, two_gamma, dy, extra, N, H, s, dmask);
    case 64: return conv32_dispatch_w<64, MODE>(W, xin, out, mask, w, bias, h, two_gamma, dy, extra, N, H, s, dmask);
  }
  return fail(ASR_E_UNSUPPORTED, "conv f32 (MFMA): C=%d", C);
}

// k_wgrad32's grid = its slab rows (one [dW | db] slab per workgroup)
template <int C, int W>
static int wgrad32_grid(int N, int H) {
  const long items = (long)N * ((H + 3) / 4);
  int cus = cu_count();
  if (cus <= 0) cus = 256;
  const int per_cu = std::max(1, std::min(2, (int)((160 * 1024) / wgrad32_lds<C, W>())));
  // at least minb bands per workgroup at C = 32 / 64: a slab row is 37 / 148 KB, written and read back
  constexpr int minb = C == 64 ? 16 : C == 32 ? 8 : 1;  // (profiles/r05al_f32_wgrad_rows_ab.txt)
  return (int)std::max<long>(1, std::min<long>({(items + minb - 1) / minb, (long)per_cu * cus, 512L}));
}

template <int C, int W, typename Tx = float>
static int launch_wgrad32(const Tx* x, const Tx* dz, int N, int H, float* slabs, int* nslabs, hipStream_t s,
                          const uint8_t* dmask = nullptr, float dh = 1.f, int layers = 1, long x_stride = 0,
                          long dz_stride = 0, long m_stride = 0, long s_stride = 0) {
  const size_t lds = wgrad32_lds<C, W>();
  const int grid = wgrad32_grid<C, W>(N, H);
  hipLaunchKernelGGL((k_wgrad32<C, W, Tx>), dim3(grid, layers), dim3(768), lds, s, x, dz, N, H, slabs, dmask, dh,
                     x_stride, dz_stride, m_stride, s_stride);
  ASR_LAUNCH_CHECK("k_wgrad32");
  *nslabs = grid;
  return ASR_OK;
}

template <typename Tin, typename Tout, int MODE>
static int launch_conv_f32(const void* xin, void* out, uint8_t* mask, const float* w, const float* bias, float h,
                           float two_gamma, const float* dy, const float* extra, int N, int H, int W, int Ci, int Co,
                           hipStream_t s, int K = 3) {
  const long tasks = (long)N * H * ((W + 15) / 16) * ((Co + 15) / 16);
  const long blocks = (tasks + 3) / 4;
  if (blocks > 0x7fffffffL) return fail(ASR_E_ARG, "conv f32: problem too large");
  if (MODE == F_EULER && mask) {
    const long bytes = ((long)N * H * W * Co + 31) / 32 * 4;
    ASR_TRY(hip_check(hipMemsetAsync(mask, 0, bytes, s), "hipMemsetAsync(mask)"));
  }
  hipLaunchKernelGGL((k_conv_f32<Tin, Tout, MODE>), dim3((unsigned)blocks), dim3(256), 0, s, (const Tin*)xin,
                     (Tout*)out, (uint32_t*)mask, w, bias, h, two_gamma, dy, extra, N, H, W, Ci, Co, K);
  ASR_LAUNCH_CHECK("k_conv_f32");
  return ASR_OK;
}

int conv_f32(int fmode, const void* xin, void* out, uint8_t* mask, const float* w, const float* bias, float h,
             float two_gamma, const float* dy, int N, int H, int W, int Ci, int Co, int out_bf16, hipStream_t s,
             const float* extra) {
  if (conv32_supported(W, Ci, Co) && fmode != F_RELU) {  // the network's blocks: fp32 MFMA
    switch (fmode) {
      case F_EULER: return conv32_dispatch<F_EULER>(Ci, W, xin, out, mask, w, bias, h, two_gamma, dy, extra, N, H, s);
      case F_CONV: return conv32_dispatch<F_CONV>(Ci, W, xin, out, mask, w, bias, h, two_gamma, dy, extra, N, H, s);
      case B_EULER: return conv32_dispatch<B_EULER>(Ci, W, xin, out, mask, w, bias, h, two_gamma, dy, extra, N, H, s);
      case B_CONV: return conv32_dispatch<B_CONV>(Ci, W, xin, out, mask, w, bias, h, two_gamma, dy, extra, N, H, s);
    }
  }
  switch (fmode) {
    case F_EULER:
      return launch_conv_f32<float, float, F_EULER>(xin, out, mask, w, bias, h, two_gamma, dy, extra, N, H, W, Ci, Co, s);
    case F_CONV:
      return launch_conv_f32<float, float, F_CONV>(xin, out, mask, w, bias, h, two_gamma, dy, extra, N, H, W, Ci, Co, s);
    case F_RELU:
      if (out_bf16)
        return launch_conv_f32<float, bf16, F_RELU>(xin, out, mask, w, bias, h, two_gamma, dy, extra, N, H, W, Ci, Co, s);
      return launch_conv_f32<float, float, F_RELU>(xin, out, mask, w, bias, h, two_gamma, dy, extra, N, H, W, Ci, Co, s);
    case B_EULER:
      return launch_conv_f32<float, float, B_EULER>(xin, out, mask, w, bias, h, two_gamma, dy, extra, N, H, W, Ci, Co, s);
    case B_CONV:
      return launch_conv_f32<float, float, B_CONV>(xin, out, mask, w, bias, h, two_gamma, dy, extra, N, H, W, Ci, Co, s);
  }
  return fail(ASR_E_ARG, "conv f32: bad mode");
}

// K x K (odd K != 3: Conv2DAntisymmetric(kernel_size), …Conv2DAntisymmetric.py:60-68, 109-145) on the
// fp32 VALU kernel, same modes as conv_f32
int conv_f32_k(int fmode, int K, const void* xin, void* out, uint8_t* mask, const float* w, const float* bias, float h,
               float two_gamma, const float* dy, int N, int H, int W, int C, hipStream_t s, const float* extra) {
  if (K == 3) return conv_f32(fmode, xin, out, mask, w, bias, h, two_gamma, dy, N, H, W, C, C, 0, s, extra);
  switch (fmode) {
    case F_EULER:
      return launch_conv_f32<float, float, F_EULER>(xin, out, mask, w, bias, h, two_gamma, dy, extra, N, H, W, C, C, s, K);
    case F_CONV:
      return launch_conv_f32<float, float, F_CONV>(xin, out, mask, w, bias, h, two_gamma, dy, extra, N, H, W, C, C, s, K);
    case B_EULER:
      return launch_conv_f32<float, float, B_EULER>(xin, out, mask, w, bias, h, two_gamma, dy, extra, N, H, W, C, C, s, K);
    case B_CONV:
      return launch_conv_f32<float, float, B_CONV>(xin, out, mask, w, bias, h, two_gamma, dy, extra, N, H, W, C, C, s, K);
  }
  return fail(ASR_E_ARG, "conv f32 (k=%d): bad mode", K);
}

int make_dz(int fmode, const void* dy, const uint8_t* mask, const void* relu_src, float h, int N, int H, int W, int C,
            int src_bf16, float* dz, hipStream_t s) {
  const long P = (long)N * H * W * C;
  const unsigned grid = (unsigned)std::min<long>((P + 255) / 256, 8192);
  if (src_bf16)
    hipLaunchKernelGGL(k_make_dz<bf16>, dim3(grid), dim3(256), 0, s, (const bf16*)dy, mask, (const bf16*)relu_src,
                       fmode, h, N, H, W, C, dz);
  else
    hipLaunchKernelGGL(k_make_dz<float>, dim3(grid), dim3(256), 0, s, (const float*)dy, mask,
                       (const float*)relu_src, fmode, h, N, H, W, C, dz);
  ASR_LAUNCH_CHECK("k_make_dz");
  return ASR_OK;
}

// The fp32 Euler block's backward on the matrix cores without the dz pass:
// dgrad (B_EULER, or B_CONV when skip_dy: the second RK2 stage) and the weight
// gradient stage dz = h dy [relu bit] straight from dy and the mask.  Only for
// conv32_supported shapes (else ASR_E_UNSUPPORTED: the caller runs make_dz +
// conv_f32 + wgrad_f32).
bool conv32_fused_bwd_supported(int W, int C) { return conv32_supported(W, C, C); }

int conv32_bwd_fused(const float* dy, const uint8_t* mask, float h, const float* x, const float* w, float two_gamma,
                     const float* extra, bool skip_dy, int N, int H, int W, int C, float* dx, bool need_w,
                     float* slabs, int* nslabs, hipStream_t s) {
  if (!conv32_supported(W, C, C)) return fail(ASR_E_UNSUPPORTED, "conv f32 fused backward: C=%d W=%d", C, W);
  *nslabs = 0;
  if (dx) {
    if (skip_dy)
      ASR_TRY(conv32_dispatch<B_CONV>(C, W, dy, dx, nullptr, w, nullptr, h, two_gamma, nullptr, extra, N, H, s, mask));
    else
      ASR_TRY(conv32_dispatch<B_EULER>(C, W, dy, dx, nullptr, w, nullptr, h, two_gamma, dy, extra, N, H, s, mask));
  }
  if (!need_w) return ASR_OK;
#define ASR_WG32F(CC)                                                                         \
  switch (W) {                                                                                \
    case 32: return launch_wgrad32<CC, 32>(x, dy, N, H, slabs, nslabs, s, mask, h);           \
    case 16: return launch_wgrad32<CC, 16>(x, dy, N, H, slabs, nslabs, s, mask, h);           \
    case 8: return launch_wgrad32<CC, 8>(x, dy, N, H, slabs, nslabs, s, mask, h);             \
  }                                                                                           \
  break
  switch (C) {
    case 16: ASR_WG32F(16);
    case 32: ASR_WG32F(32);
    case 64: ASR_WG32F(64);
  }
#undef ASR_WG32F
  return fail(ASR_E_UNSUPPORTED, "conv f32 fused backward: C=%d W=%d", C, W);
}

// number of row chunks used by the fp32 wgrad (bounded by kMaxSlabs in the
// workspace sizing of the callers)
int wgrad_f32_chunks(int N, int H) {
  const long R = (long)N * H;
  long chunks = std::min<long>(R, 256);
  return (int)std::max<long>(chunks, 1);
}

// Slab rows one fp32 3x3 C -> C block application's weight gradient writes
// (conv32_bwd_fused / wgrad_f32): the workspace of the fp32 networks keeps
// every block's slabs, so it is sized by this, not by the 512-row maximum.
// On the device the workspace was sized for (the MFMA grid follows its CU count).
int f32_block_slab_rows(int N, int H, int W, int C) {
  if (conv32_supported(W, C, C)) {
#define ASR_WR(CC)                                      \
  switch (W) {                                          \
    case 32: return wgrad32_grid<CC, 32>(N, H);         \
    case 16: return wgrad32_grid<CC, 16>(N, H);         \
    case 8: return wgrad32_grid<CC, 8>(N, H);           \
  }                                                     \
  break
    switch (C) {
      case 16: ASR_WR(16);
      case 32: ASR_WR(32);
      case 64: ASR_WR(64);
    }
#undef ASR_WR
  }
  return wgrad_f32_chunks(N, H);
}

int wgrad_f32(const void* x, int x_bf16, const float* dz, int N, int H, int W, int Ci, int Co, float* slabs,
              int* nslabs, hipStream_t s, int K) {
  if (!x_bf16 && K == 3 && conv32_supported(W, Ci, Co)) {  // the network's blocks: fp32 MFMA, db included
#define ASR_WG32(CC)                                                                         \
  switch (W) {                                                                               \
    case 32: return launch_wgrad32<CC, 32>((const float*)x, dz, N, H, slabs, nslabs, s);     \
    case 16: return launch_wgrad32<CC, 16>((const float*)x, dz, N, H, slabs, nslabs, s);     \
    case 8: return launch_wgrad32<CC, 8>((const float*)x, dz, N, H, slabs, nslabs, s);       \
  }                                                                                          \
  break
    switch (Ci) {
      case 16: ASR_WG32(16);
      case 32: ASR_WG32(32);
      case 64: ASR_WG32(64);
    }
#undef ASR_WG32
  }
  const long R = (long)N * H;
  const int chunks = wgrad_f32_chunks(N, H);
  const int rpc = (int)((R + chunks - 1) / chunks);
  const int nch = (int)((R + rpc - 1) / rpc);
  const long E = (long)K * K * Ci * Co;
  dim3 grid((unsigned)((E + 255) / 256), nch);
  if (x_bf16)
    hipLaunchKernelGGL(k_wgrad_f32<bf16>, grid, dim3(256), 0, s, (const bf16*)x, dz, N, H, W, Ci, Co, rpc, slabs, K);
  else
    hipLaunchKernelGGL(k_wgrad_f32<float>, grid, dim3(256), 0, s, (const float*)x, dz, N, H, W, Ci, Co, rpc, slabs, K);
  ASR_LAUNCH_CHECK("k_wgrad_f32");
  if (Co > 1024) return fail(ASR_E_UNSUPPORTED, "db: C > 1024");
  hipLaunchKernelGGL(k_db_f32, dim3(nch), dim3(((Co + 63) / 64) * 64), 0, s, dz, R, W, Co, rpc, E, slabs);
  ASR_LAUNCH_CHECK("k_db_f32");
  *nslabs = nch;
  return ASR_OK;
}

// ===========================================================================
// bf16 block kernels at any stage width (W in {32, 16, 8}, C in {16, 32, 64}):
// the multi-stage nets' identity blocks in bf16 (the He-style ResNet-32 at the
// metric's precision, tfkeras_resnets.py:575-593).  k_conv32's geometry on
// v_mfma_f32_16x16x32_bf16: a workgroup (4 waves) owns a band of BR = 4 output
// rows of one image, the BR + 2 input rows staged in LDS as bf16 (pixel-major,
// C channels contiguous; zero rows outside the image and zero halo columns),
// every wave keeps its o-tile's A = W^T fragments (asr_theta_to_w's bf16 pack:
// lane (lx, g) holds W^T[16 ot + lx][32 ks + 8 g .. + 7]) in registers and walks
// its share of the band's 16-pixel tiles.  B fragment of k-step ks, lane (lx, g):
// kappa = 32 ks + 8 g .. + 7 = tap t, channels i0 .. i0 + 7 of the pixel shifted
// by t: one 16-B LDS read.  The accumulator lane (lx, g) holds channels 4g..4g+3
// of pixel lx, as in the fp32 kernel (the same epilogue and mask nibbles).
//   F_EULER: y = x + h relu(conv(x) + b), relu-mask bits;
//   B_EULER: the tile holds dz = dy & mask (exact), dx = dy - h conv(dz) + 2 gamma h dz.
// The weight gradient runs k_wgrad32 on the bf16 operands (staged to fp32 in
// LDS, fp32 MFMA: the reduction is in fp32 either way, as the bf16 stacks').
// ===========================================================================
template <int C, int W_>
struct BfBand {
  // PS: a pixel's elements in the LDS tiles, padded so the 16 lanes of a 16-B read (16 consecutive
  // pixels) fall on distinct banks (unpadded, C = 64 put them on 2 bank groups: 8-way conflicts)
  static constexpr int OT = C / 16, W = W_, TW = W + 2, BR = 4, PS = C + 8, TILEE = (BR + 2) * TW * PS;
  static constexpr int T = BR * W / 16;  // 16-pixel tiles per band
  static constexpr int WPT = 4 / OT;     // waves sharing an o-tile
  static constexpr int KS = (9 * C + 31) / 32;
  static_assert(W == 8 || W == 16 || W == 32, "bf16 band: W in {8, 16, 32}");
};

// 8 bf16 masked by 8 relu bits (bit j -> halfword j)
__device__ __forceinline__ uint4 mask8_bf16(uint4 v, unsigned bits) {
  auto h2 = [&](unsigned b) { return ((b & 1u) ? 0xffffu : 0u) | ((b & 2u) ? 0xffff0000u : 0u); };
  v.x &= h2(bits);
  v.y &= h2(bits >> 2);
  v.z &= h2(bits >> 4);
  v.w &= h2(bits >> 6);
  return v;
}

template <int C, int W, int MODE>
__global__ __launch_bounds__(256) void k_convb(const bf16* __restrict__ xin, bf16* __restrict__ out,
                                               uint8_t* __restrict__ mask, const bf16* __restrict__ wpack,
                                               const float* __restrict__ bias, float h, float two_gamma,
                                               const bf16* __restrict__ dy, int N, int H,
                                               const uint8_t* __restrict__ dmask) {
  using G = BfBand<C, W>;
  constexpr int OT = G::OT, TW = G::TW, BR = G::BR, KS = G::KS, C8 = C / 8;
  constexpr int NCH = (BR + 2) * TW * C8, NPT = (NCH + 255) / 256;
  __shared__ __attribute__((aligned(16))) bf16 tile[G::TILEE];
  // backward: the band's own rows of dy unmasked (the epilogue's dy term), beside the dz tile
  __shared__ __attribute__((aligned(16))) bf16 dyc[MODE == B_EULER ? BR * W * G::PS : 8];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, lx = lane & 15;
  const int ot = wave % OT, rw = wave / OT;
  const int nb = (H + BR - 1) / BR;
  const long items = (long)N * nb;
  // persistent: a run of bands per workgroup, the W fragments loaded once, the next band's rows
  // in registers while this band's MFMAs run
  const long i0 = (long)blockIdx.x * items / gridDim.x, i1 = (long)(blockIdx.x + 1) * items / gridDim.x;
  bf16x8 A[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) A[ks] = *(const bf16x8*)(wpack + (((long)ot * KS + ks) * 64 + lane) * 8);
  f32x4 bz = {0.f, 0.f, 0.f, 0.f};
  if ((MODE == F_EULER || MODE == F_CONV) && bias) bz = *(const f32x4*)(bias + 16 * ot + 4 * g);
  uint4 pf[NPT];
  unsigned pm[NPT];
  auto fetch = [&](long item) {
    const int n = (int)(item / nb), y0 = (int)(item % nb) * BR;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int i = tid + 256 * k;
      const int r = i / (TW * C8), rem = i % (TW * C8), col = rem / C8, c8 = rem % C8;
      const int gy = y0 - 1 + r, gx = col - 1;
      pf[k] = make_uint4(0u, 0u, 0u, 0u);
      pm[k] = 0u;
      if (i < NCH && (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W) {
        const long e = (((long)n * H + gy) * W + gx) * C + 8 * c8;
        pf[k] = *(const uint4*)(xin + e);
        if (MODE == B_EULER) pm[k] = dmask[e >> 3];
      }
    }
  };
  if (i0 < i1) fetch(i0);
  for (long item = i0; item < i1; ++item) {
    const int n = (int)(item / nb), y0 = (int)(item % nb) * BR;
    __syncthreads();  // the previous band's tile consumed
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int i = tid + 256 * k;
      if (i >= NCH) break;
      const int r = i / (TW * C8), rem = i % (TW * C8), col = rem / C8, c8 = rem % C8;
      bf16* dst = tile + (r * TW + col) * G::PS + 8 * c8;
      if constexpr (MODE == B_EULER) {  // the tile gets dz = dy & mask; the band's rows keep dy
        *(uint4*)dst = mask8_bf16(pf[k], pm[k]);
        if (r >= 1 && r <= BR && col >= 1 && col <= W) *(uint4*)(dyc + ((r - 1) * W + col - 1) * G::PS + 8 * c8) = pf[k];
      } else {
        *(uint4*)dst = pf[k];
      }
    }
    __syncthreads();
    if (item + 1 < i1) fetch(item + 1);
    constexpr int NT = (G::T + G::WPT - 1) / G::WPT;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int tau = rw + j * G::WPT;
      if (tau >= G::T) break;  // (wave-uniform)
      const int bp = 16 * tau + lx, r = bp / W, px = bp % W;
      if (W >= 16 && y0 + r >= H) break;  // (wave-uniform for W >= 16; rows only grow with tau)
      f32x4 acc = bz;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int kap = 32 * ks + 8 * g;
        const int t = min(kap / C, 8), i0c = kap - (kap / C) * C;  // (C = 16, last k-step: tap 9 pads A with zeros)
        const uint4 bv = *(const uint4*)(tile + ((r + t / 3) * TW + px + t % 3) * G::PS + i0c);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[ks], __builtin_bit_cast(bf16x8, bv), acc, 0, 0, 0);
      }
      mfma_bf16_settle();  // (the epilogue branches: every path must see the result's wait states)
      const bool ok = y0 + r < H;
      const long pix = ((long)n * H + y0 + r) * W + px;
      const long oi = pix * C + 16 * ot + 4 * g;  // this lane's 4 channels
      const uint2 cw = *(const uint2*)(tile + ((r + 1) * TW + px + 1) * G::PS + 16 * ot + 4 * g);  // x or dz at the pixel
      const float ctr[4] = {__uint_as_float(cw.x << 16), __uint_as_float(cw.x & 0xffff0000u),
                            __uint_as_float(cw.y << 16), __uint_as_float(cw.y & 0xffff0000u)};
      float v[4];
      if constexpr (MODE == F_EULER) {
        unsigned nib = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float z = acc[e];
          nib |= (z > 0.f ? 1u : 0u) << e;
          v[e] = fmaf(h, fmaxf(z, 0.f), ctr[e]);
        }
        if (mask) {  // the pixel's 16 channels of this o-tile: 4 nibbles, one 16-bit store
          unsigned m = nib << (4 * g);
          m |= (unsigned)__shfl_xor((int)m, 16, 64);
          m |= (unsigned)__shfl_xor((int)m, 32, 64);
          if (g == 0 && ok) *(uint16_t*)(mask + (pix * C + 16 * ot) / 8) = (uint16_t)m;
        }
      } else if constexpr (MODE == F_CONV) {  // the bare layer call: z = conv(x, W) + b
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[e];
      } else if constexpr (MODE == B_CONV) {  // its backward: dz = dy (the tile), dx = A^T dz = -A dz + 2 gamma dz
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaf(two_gamma, ctr[e], -acc[e]);
      } else {  // B_EULER: the tile holds dz = dy & mask
        const uint2 dw = *(const uint2*)(dyc + (r * W + px) * G::PS + 16 * ot + 4 * g);
        const float d0[4] = {__uint_as_float(dw.x << 16), __uint_as_float(dw.x & 0xffff0000u),
                             __uint_as_float(dw.y << 16), __uint_as_float(dw.y & 0xffff0000u)};
        const float hg = h * two_gamma;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaf(hg, ctr[e], fmaf(-h, acc[e], d0[e]));
      }
      if (ok) *(uint2*)(out + oi) = make_uint2(pk_bf16_rn(v[0], v[1]), pk_bf16_rn(v[2], v[3]));
    }
  }
}

bool convb_supported(int W, int C) { return (W == 32 || W == 16 || W == 8) && (C == 16 || C == 32 || C == 64); }

template <int C, int W, int MODE>
static int launch_convb(const bf16* xin, bf16* out, uint8_t* mask, const bf16* w, const float* bias, float h,
                        float two_gamma, const bf16* dy, int N, int H, const uint8_t* dmask, hipStream_t s) {
  const long items = (long)N * ((H + 3) / 4);
  int cus = cu_count();
  if (cus <= 0) cus = 256;
  const long grid = std::max<long>(1, std::min<long>(items, 4L * cus));  // 4 persistent workgroups per CU (r05r)
  hipLaunchKernelGGL((k_convb<C, W, MODE>), dim3((unsigned)grid), dim3(256), 0, s, xin, out, mask, w, bias, h,
                     two_gamma, dy, N, H, dmask);
  ASR_LAUNCH_CHECK("k_convb");
  return ASR_OK;
}

// ---------------------------------------------------------------------------
// The bf16 weight gradient at any stage width on v_mfma_f32_16x16x32_bf16
// (k_wgradb): D[t][i][o] = h sum_px x[px + tap t][i] dz[px][o], dz = dy & mask
// (exact in bf16; h applied to the fp32 sums), db[o] = h sum_px dz[px][o].
// K = pixels: a workgroup stages a band of BR = 128 / W rows of one image (x
// with its halo rows / columns, dz) in LDS, pixel-major with C channels
// contiguous, and reads both operands with ds_read_b64_tr_b16 (T10): a 16-lane
// group's lane (q, p) addresses pixel q of 4, channels 4p .. 4p+3, and lane lx
// receives channel lx of the 4 pixels -- the MFMA fragment's k run.  A 32-pixel
// chunk's k order is permuted the same way in both operands: lane group g takes
// pixels 4g .. 4g+3 (first read) and 16 + 4g .. (second), so a 32-lane half
// reads 8 consecutive pixels.  The 16-B chunk c of pixel P sits at chunk
// c ^ f(P) (f = 2 ((P >> 1) & 3) at C = 64, 2 ((P >> 2) & 1) at C = 32, 0 at
// C = 16): the half's 8 pixels x 32 B then cover all 64 banks.
// Waves: TS pair splits (i-tile it, NO o-tiles: the 9 taps' A fragments feed
// NO MFMAs each) x PS chunk splits, partials summed through LDS at the end;
// db on MFMA (ones x dz) in the it = 0 waves.  Persistent over bands, the next
// band's global loads in flight during this band's MFMAs (dz = dy & mask formed
// at the LDS store, so nothing waits for them before); one [dW | db] slab
// per workgroup, the rows the fp32 wgrad grid sizes (f32_block_slab_rows).
// ---------------------------------------------------------------------------
template <int C, int W_>
struct WgB {
  static constexpr int OT = C / 16, W = W_, TW = W + 2, BR = 128 / W;
  static constexpr int NO = C == 16 ? 1 : 2, TS = OT * (OT / NO), PS = C == 64 ? 1 : 4, NW = TS * PS, NTH = 64 * NW;
  static constexpr int C8 = C / 8, XCH = (BR + 2) * TW * C8, DCH = BR * W * C8;
  static constexpr int XPT = (XCH + NTH - 1) / NTH, DPT = (DCH + NTH - 1) / NTH;
  static constexpr int XE = (BR + 2) * TW * C, DE = BR * W * C;
  static constexpr int ACC = (9 + 1) * NO;  // accumulator tiles per wave (9 taps + db per o-tile)
  static constexpr size_t LDS = (size_t)(XE + DE) * 2 + (PS > 1 ? (size_t)TS * ACC * 256 * 4 : 0);
  static_assert(W == 8 || W == 16 || W == 32, "bf16 wgrad: W in {8, 16, 32}");
  __host__ __device__ static constexpr int swz(int P) {
    return C == 64 ? 2 * ((P >> 1) & 3) : C == 32 ? 2 * ((P >> 2) & 1) : 0;
  }
};

// one transposed-read k run: 4 pixels' 4 channels -> the lane's 4 bf16 of one channel
__device__ __forceinline__ s16x4 tr4(const bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((ASR_LDS s16x4*)p);
}

// MASKED false: dz = dy (the bare conv's weight gradient, B_CONV; dmask unused)
template <int C, int W, bool MASKED = true>
__global__ __launch_bounds__((WgB<C, W>::NTH)) void k_wgradb(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                           const uint8_t* __restrict__ dmask, int N, int H, float h,
                                                           float* __restrict__ slabs, long x_stride, long dy_stride,
                                                           long m_stride, long s_stride) {
  using G = WgB<C, W>;
  // several layers in one launch: blockIdx.y is the layer (strides in elements / bytes / floats)
  x += blockIdx.y * x_stride;
  dy += blockIdx.y * dy_stride;
  dmask += blockIdx.y * m_stride;
  slabs += blockIdx.y * s_stride;
  constexpr int TW = G::TW, BR = G::BR, NO = G::NO, OT = G::OT, E = 9 * C * C;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_wb[];
  bf16* xt = (bf16*)lds_wb;               // [BR+2][TW][C] (chunk-swizzled per pixel)
  bf16* dzt = xt + G::XE;                 // [BR][W][C]
  float* red = (float*)(dzt + G::DE);     // [TS][ACC][64][4] (PS > 1)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, lx = lane & 15;
  const int q = lx >> 2, pq = lx & 3;
  const int ts = wave % G::TS, ps = wave / G::TS;
  const int it = ts / (OT / NO), ob = (ts % (OT / NO)) * NO;
  const int nb = (H + BR - 1) / BR;
  const long items = (long)N * nb;
  const long i0 = (long)blockIdx.x * items / gridDim.x, i1 = (long)(blockIdx.x + 1) * items / gridDim.x;
  f32x4 acc[9][NO], accb[NO];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int o = 0; o < NO; ++o) acc[t][o] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int o = 0; o < NO; ++o) accb[o] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint4 px[G::XPT], pd[G::DPT];
  unsigned pm[G::DPT];  // the relu bits, applied at the LDS store: masking here would wait for the loads
  auto fetch = [&](long item) {
    const int n = (int)(item / nb), y0 = (int)(item % nb) * BR;
#pragma unroll
    for (int k = 0; k < G::XPT; ++k) {
      const int i = tid + k * G::NTH;
      px[k] = make_uint4(0u, 0u, 0u, 0u);
      const int r = i / (TW * G::C8), rem = i % (TW * G::C8), col = rem / G::C8, c8 = rem % G::C8;
      const int gy = y0 - 1 + r, gx = col - 1;
      if (i < G::XCH && (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W)
        px[k] = *(const uint4*)(x + (((long)n * H + gy) * W + gx) * C + 8 * c8);
    }
#pragma unroll
    for (int k = 0; k < G::DPT; ++k) {
      const int i = tid + k * G::NTH;
      pd[k] = make_uint4(0u, 0u, 0u, 0u);
      pm[k] = 0u;
      const int r = i / (W * G::C8);
      if (i < G::DCH && y0 + r < H) {
        const long e = ((long)n * H + y0) * W * C + 8L * i;
        pd[k] = *(const uint4*)(dy + e);
        if constexpr (MASKED) pm[k] = dmask[e >> 3];
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int k = 0; k < G::XPT; ++k) {
      const int i = tid + k * G::NTH;
      const int P = i / G::C8, c8 = i % G::C8;
      if (i < G::XCH) *(uint4*)(xt + P * C + 8 * (c8 ^ G::swz(P))) = px[k];
    }
#pragma unroll
    for (int k = 0; k < G::DPT; ++k) {
      const int i = tid + k * G::NTH;
      const int P = i / G::C8, c8 = i % G::C8;
      if (i < G::DCH) *(uint4*)(dzt + P * C + 8 * (c8 ^ G::swz(P))) = MASKED ? mask8_bf16(pd[k], pm[k]) : pd[k];
    }
  };
  // the lane's 8-B piece of channels 16 ch + 4 pq .. +3 at pixel P of a tile
  auto piece = [&](const bf16* tile, int P, int ch) {
    const int c16 = 2 * ch + (pq >> 1);
    return tile + P * C + 8 * (c16 ^ G::swz(P)) + 4 * (pq & 1);
  };
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  auto frag = [&](const bf16* tile, int P1, int P2, int ch) {
    const s16x4 a = tr4(piece(tile, P1, ch)), b = tr4(piece(tile, P2, ch));
    const s16x8 c = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    return __builtin_bit_cast(bf16x8, c);
  };
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (bf16)1.f;
  if (i0 < i1) fetch(i0);
  for (long item = i0; item < i1; ++item) {
    const int y0 = (int)(item % nb) * BR;
    const int rows = min(BR, H - y0), nch = (rows * W + 31) / 32;
    __syncthreads();  // the previous band's operands consumed
    store();
    __syncthreads();
    if (item + 1 < i1) fetch(item + 1);  // in flight during this band's MFMAs
    for (int ch = ps; ch < nch; ch += G::PS) {  // (wave-uniform: EXEC stays full for the transposed reads)
      const int k1 = 32 * ch + 4 * g + q, k2 = k1 + 16;
      const int r1 = k1 / W, c1 = k1 % W, r2 = k2 / W, c2 = k2 % W;
      bf16x8 B[NO];
#pragma unroll
      for (int o = 0; o < NO; ++o) B[o] = frag(dzt, r1 * W + c1, r2 * W + c2, ob + o);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int d = (t / 3) * TW + t % 3;
        const bf16x8 A = frag(xt, r1 * TW + c1 + d, r2 * TW + c2 + d, it);
#pragma unroll
        for (int o = 0; o < NO; ++o) acc[t][o] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, B[o], acc[t][o], 0, 0, 0);
      }
      if (it == 0) {
#pragma unroll
        for (int o = 0; o < NO; ++o) accb[o] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, B[o], accb[o], 0, 0, 0);
      }
    }
  }
  // the PS chunk-split partials, summed in a fixed order through LDS (one split at a time)
  if constexpr (G::PS > 1) {
    float* mine = red + (long)ts * G::ACC * 256;
#pragma unroll 1
    for (int src = 1; src < G::PS; ++src) {
      __syncthreads();
      if (ps == src) {
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
          for (int o = 0; o < NO; ++o) *(f32x4*)(mine + ((t * NO + o) * 64 + lane) * 4) = acc[t][o];
#pragma unroll
        for (int o = 0; o < NO; ++o) *(f32x4*)(mine + ((9 * NO + o) * 64 + lane) * 4) = accb[o];
      }
      __syncthreads();
      if (ps == 0) {
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
          for (int o = 0; o < NO; ++o) acc[t][o] += *(const f32x4*)(mine + ((t * NO + o) * 64 + lane) * 4);
#pragma unroll
        for (int o = 0; o < NO; ++o) accb[o] += *(const f32x4*)(mine + ((9 * NO + o) * 64 + lane) * 4);
      }
    }
  }
  if (ps == 0) {
    float* slab = slabs + (long)blockIdx.x * (E + C);
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int o = 0; o < NO; ++o)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          slab[((long)t * C + 16 * it + 4 * g + e) * C + 16 * (ob + o) + lx] = h * acc[t][o][e];
    if (it == 0 && g == 0) {
#pragma unroll
      for (int o = 0; o < NO; ++o) slab[E + 16 * (ob + o) + lx] = h * accb[o][0];
    }
  }
}

template <int C, int W, bool MASKED = true>
static int launch_wgradb(const bf16* x, const bf16* dy, const uint8_t* mask, int N, int H, float h, float* slabs,
                         int* nslabs, hipStream_t s, int layers = 1, long x_stride = 0, long dy_stride = 0,
                         long m_stride = 0, long s_stride = 0) {
  using G = WgB<C, W>;
  const long items = (long)N * ((H + G::BR - 1) / G::BR);
  // at most the fp32 wgrad's grid: the rows the workspaces size per block (f32_block_slab_rows)
  // bands per workgroup (profiles/r05_he32_bf16_ab.txt; re-measured after this round's reductions:
  // profiles/r06ai_wgradb_grid_ab.txt)
  constexpr int minb = C == 16 ? 1 : C == 32 ? 8 : 32;
  const int grid = (int)std::max<long>(1, std::min<long>((items + minb - 1) / minb, wgrad32_grid<C, W>(N, H)));
  hipLaunchKernelGGL((k_wgradb<C, W, MASKED>), dim3(grid, layers), dim3(G::NTH), G::LDS, s, x, dy, mask, N, H, h, slabs,
                     x_stride, dy_stride, m_stride, s_stride);
  ASR_LAUNCH_CHECK("k_wgradb");
  *nslabs = grid;
  return ASR_OK;
}

// y = x + h relu(conv(x, W) + b) in bf16 (w: asr_theta_to_w's ASR_BF16 pack of one layer); with
// conv_only the bare layer call y = conv(x, W) + b (…3By3.py:157-171; no mask, h unused)
int convb_forward(const void* x, void* y, uint8_t* mask, const void* w, const float* bias, float h, int N, int H, int W,
                  int C, hipStream_t s, bool conv_only) {
#define ASR_CB(CC, WW)                                                                                              \
  if (C == CC && W == WW) {                                                                                         \
    if (conv_only)                                                                                                  \
      return launch_convb<CC, WW, F_CONV>((const bf16*)x, (bf16*)y, nullptr, (const bf16*)w, bias, 1.f, 0.f,        \
                                          nullptr, N, H, nullptr, s);                                               \
    return launch_convb<CC, WW, F_EULER>((const bf16*)x, (bf16*)y, mask, (const bf16*)w, bias, h, 0.f, nullptr, N, H, \
                                         nullptr, s);                                                               \
  }
  ASR_CB(16, 32) ASR_CB(16, 16) ASR_CB(16, 8) ASR_CB(32, 32) ASR_CB(32, 16) ASR_CB(32, 8) ASR_CB(64, 32)
  ASR_CB(64, 16) ASR_CB(64, 8)
#undef ASR_CB
  return fail(ASR_E_UNSUPPORTED, "conv bf16 (any width): C=%d W=%d", C, W);
}

// The Euler block's backward in bf16: dx = dy - h conv(dy & mask, W) + 2 gamma h (dy & mask)
// (W: the forward pack for antisymmetric operators, whose transpose is -A + 2 gamma I; the
// transposed operator's pack with gamma = 0 otherwise) and the weight-gradient slabs
// (k_wgradb on the bf16 x and dz = dy & mask, h on the fp32 sums).  conv_only: the bare layer
// call's backward, dz = dy: dx = -conv(dy, W) + 2 gamma dy, slabs of x (x) dy (h unused)
int convb_backward(const void* dy, const uint8_t* mask, const void* x, const void* w, float h, float two_gamma, int N,
                   int H, int W, int C, void* dx, bool need_w, float* slabs, int* nslabs, hipStream_t s,
                   bool conv_only) {
  *nslabs = 0;
  if (!convb_supported(W, C)) return fail(ASR_E_UNSUPPORTED, "conv bf16 backward (any width): C=%d W=%d", C, W);
  if (dx) {
#define ASR_CB(CC, WW)                                                                                                  \
  if (C == CC && W == WW) {                                                                                             \
    if (conv_only)                                                                                                      \
      ASR_TRY((launch_convb<CC, WW, B_CONV>((const bf16*)dy, (bf16*)dx, nullptr, (const bf16*)w, nullptr, 1.f,        \
                                            two_gamma, nullptr, N, H, nullptr, s)));                                   \
    else                                                                                                                \
      ASR_TRY((launch_convb<CC, WW, B_EULER>((const bf16*)dy, (bf16*)dx, nullptr, (const bf16*)w, nullptr, h,         \
                                             two_gamma, (const bf16*)dy, N, H, mask, s)));                             \
  }
    ASR_CB(16, 32) ASR_CB(16, 16) ASR_CB(16, 8) ASR_CB(32, 32) ASR_CB(32, 16) ASR_CB(32, 8) ASR_CB(64, 32)
    ASR_CB(64, 16) ASR_CB(64, 8)
#undef ASR_CB
  }
  if (!need_w) return ASR_OK;
#define ASR_WB(CC, WW)                                                                                             \
  if (C == CC && W == WW) {                                                                                        \
    if (conv_only)                                                                                                 \
      return launch_wgradb<CC, WW, false>((const bf16*)x, (const bf16*)dy, nullptr, N, H, 1.f, slabs, nslabs, s); \
    return launch_wgradb<CC, WW>((const bf16*)x, (const bf16*)dy, mask, N, H, h, slabs, nslabs, s);              \
  }
  ASR_WB(16, 32) ASR_WB(16, 16) ASR_WB(16, 8) ASR_WB(32, 32) ASR_WB(32, 16) ASR_WB(32, 8) ASR_WB(64, 32)
  ASR_WB(64, 16) ASR_WB(64, 8)
#undef ASR_WB
  return fail(ASR_E_UNSUPPORTED, "conv bf16 backward (any width): C=%d W=%d", C, W);
}

// ===========================================================================
// Image-resident bf16 stages (k_stagef / k_stageb): all L Euler blocks of a
// 16 x 16 x 32 or 8 x 8 x 64 stage in one launch, a workgroup per image with
// the image in LDS (20.3 / 12.5 KiB with its zero halo), as the deep16 kernels
// do for 32 x 32 x 16.  The conv is k_convb's (v_mfma_f32_16x16x32_bf16, the
// layer's A fragments in registers, B one 16-B LDS read per k-step); between
// layers only LDS traffic and a barrier.
//   forward: ping-pong image buffers; each layer's y and relu mask to HBM (the
//     backward reads them), y into the other buffer;
//   backward (input gradient only): dy in LDS, dz = dy & mask_l into the halo
//     tile, dx = dy - h conv(dz) + 2 gamma h dz written over dy in place (a lane
//     reads and writes only its own pixel's channels); the gradient entering
//     each layer below the top goes to HBM for the weight gradient (k_wgradb
//     per layer, unchanged), dx_0 at the end.
// ===========================================================================
template <int C, int W_>
struct StImg {
  static constexpr int NW = 4, NTH = 64 * NW;  // waves per image
  static constexpr int W = W_, H = W_, TW = W + 2, OT = C / 16, WPT = NW / OT, KS = (9 * C + 31) / 32, C8 = C / 8;
  static constexpr int T = H * W / 16;              // 16-pixel tiles per image
  static_assert((T / WPT) % 2 == 0, "image-resident stage: a wave's tiles come in pairs (two MFMA chains)");
  static constexpr int PS = C + 8;          // a pixel's elements in LDS (padded, as BfBand)
  static constexpr int IMGE = (H + 2) * TW * PS;    // elements of a haloed image tile
  static constexpr int NCH = H * W * C8;            // 16-B chunks of an image
  static_assert((W == 16 && C == 32) || (W == 8 && C == 64) || (W == 8 && C == 32),
                "image-resident stage: 16 x 16 x 32, 8 x 8 x 32 or 8 x 8 x 64");
};

template <int C, int W>
__device__ __forceinline__ int st_off(int r, int c) {  // element offset of interior pixel (r, c) in a haloed tile
  return ((r + 1) * StImg<C, W>::TW + c + 1) * StImg<C, W>::PS;
}

// an LDS-only workgroup barrier: the layers' global stores (y, masks, dy) stay in flight across it
// (__syncthreads waits for them too: a full store round trip per layer)
__device__ __forceinline__ void st_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// an image's NCH 16-B chunks from global into LDS, put(i, v) storing chunk i: every load of a thread
// issued before its first store (a load-store loop waited for each load in turn)
template <int NCH, int NTH, typename V, typename T, typename Put>
__device__ __forceinline__ void st_fetch_image(const T* __restrict__ src, int tid, Put put) {
  constexpr int NPT = (NCH + NTH - 1) / NTH, EPC = 16 / (int)sizeof(T);
  V v[NPT];
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int i = tid + k * NTH;
    if (i < NCH) v[k] = *(const V*)(src + (long)EPC * i);
  }
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int i = tid + k * NTH;
    if (i < NCH) put(i, v[k]);
  }
}

constexpr int kStIpw = 1;
// IPW images per workgroup: 1 (a wave's two MFMA chains are two tiles of the image); 2 (the chains are
// one tile of each image, the layer's A fragments shared) measured -7 % (r05ar: half the workgroups)
template <int C, int W>
__global__ __launch_bounds__((StImg<C, W>::NTH)) void k_stagef(const bf16* __restrict__ x0, bf16* __restrict__ ys, long y_stride,
                                                uint8_t* __restrict__ masks, long mask_stride,
                                                const bf16* __restrict__ wpack, long w_stride,
                                                const float* __restrict__ bias, long bias_stride, float h, int N,
                                                int L) {
  using G = StImg<C, W>;
  constexpr int TW = G::TW, KS = G::KS, OT = G::OT, IPW = kStIpw, TP = 2 / IPW;
  extern __shared__ __attribute__((aligned(16))) bf16 lds_stf[];  // [IPW][2][IMGE]
  auto imgb = [&](int im, int pp) { return lds_stf + (im * 2 + pp) * G::IMGE; };
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, lx = lane & 15;
  const int ot = wave % OT, rw = wave / OT;
  for (int i = tid; i < IPW * 2 * G::IMGE / 8; i += G::NTH) ((uint4*)lds_stf)[i] = make_uint4(0u, 0u, 0u, 0u);
  st_barrier();
  for (int n0 = IPW * blockIdx.x; n0 < N; n0 += IPW * gridDim.x) {
    const int nimg = min(IPW, N - n0);  // (uniform)
    for (int im = 0; im < nimg; ++im) {
      const long ib = (long)(n0 + im) * G::H * W * C;
      bf16* dst = imgb(im, 0);
      st_fetch_image<G::NCH, G::NTH, uint4>(x0 + ib, tid, [&](int i, const uint4& v) {
        const int px = i / G::C8, c8 = i % G::C8;
        *(uint4*)(dst + st_off<C, W>(px / W, px % W) + 8 * c8) = v;
      });
    }
    st_barrier();
    for (int l = 0; l < L; ++l) {
      bf16x8 A[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        A[ks] = *(const bf16x8*)(wpack + (long)l * w_stride + (((long)ot * KS + ks) * 64 + lane) * 8);
      const f32x4 bz = *(const f32x4*)(bias + (long)l * bias_stride + 16 * ot + 4 * g);
      uint8_t* ml = masks + (long)l * mask_stride;
      auto epi = [&](int im, int p, const f32x4& acc) {
        const bf16* cur = imgb(im, l & 1);
        bf16* nxt = imgb(im, (l & 1) ^ 1);
        const long n = n0 + im;
        const int r = p / W, px = p % W;
        const int co = st_off<C, W>(r, px) + 16 * ot + 4 * g;
        const uint2 cw = *(const uint2*)(cur + co);
        const float ctr[4] = {__uint_as_float(cw.x << 16), __uint_as_float(cw.x & 0xffff0000u),
                              __uint_as_float(cw.y << 16), __uint_as_float(cw.y & 0xffff0000u)};
        float v[4];
        unsigned nib = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          nib |= (acc[e] > 0.f ? 1u : 0u) << e;
          v[e] = fmaf(h, fmaxf(acc[e], 0.f), ctr[e]);
        }
        const uint2 yw = make_uint2(pk_bf16_rn(v[0], v[1]), pk_bf16_rn(v[2], v[3]));
        *(uint2*)(nxt + co) = yw;
        const long pix = n * G::H * W + p;
        *(uint2*)(ys + (long)l * y_stride + pix * C + 16 * ot + 4 * g) = yw;
        unsigned m = nib << (4 * g);
        m |= (unsigned)__shfl_xor((int)m, 16, 64);
        m |= (unsigned)__shfl_xor((int)m, 32, 64);
        if (g == 0) *(uint16_t*)(ml + (pix * C + 16 * ot) / 8) = (uint16_t)m;
      };
#pragma unroll 1
      for (int j = 0; j < G::T / G::WPT; j += TP) {
        int pc[2], rc[2], xc[2];
        const bf16* bc[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {  // chain c: image c / TP, tile j + c % TP
          pc[c] = 16 * (rw + (j + c % TP) * G::WPT) + lx;
          rc[c] = pc[c] / W;
          xc[c] = pc[c] % W;
          bc[c] = imgb(c / TP, l & 1);
        }
        f32x4 acc[2] = {bz, bz};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const int kap = 32 * ks + 8 * g;
          const int t = min(kap / C, 8), i0c = kap - (kap / C) * C;
          uint4 b[2];
#pragma unroll
          for (int c = 0; c < 2; ++c)
            b[c] = *(const uint4*)(bc[c] + ((rc[c] + t / 3) * TW + xc[c] + t % 3) * G::PS + i0c);
#pragma unroll
          for (int c = 0; c < 2; ++c)
            acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[ks], __builtin_bit_cast(bf16x8, b[c]), acc[c], 0, 0, 0);
        }
        mfma_bf16_settle();
#pragma unroll
        for (int c = 0; c < 2; ++c)
          if (c / TP < nimg) epi(c / TP, pc[c], acc[c]);
      }
      st_barrier();  // layer l's outputs complete; the inputs free
    }
  }
}

template <int C, int W>
__global__ __launch_bounds__((StImg<C, W>::NTH)) void k_stageb(const bf16* __restrict__ dyL, bf16* __restrict__ dys, long d_stride,
                                                bf16* __restrict__ dx0, const uint8_t* __restrict__ masks,
                                                long mask_stride, const bf16* __restrict__ wpack, long w_stride,
                                                float h, float two_gamma, int N, int L) {
  using G = StImg<C, W>;
  constexpr int TW = G::TW, KS = G::KS, OT = G::OT, IPW = kStIpw, TP = 2 / IPW;
  constexpr int DYE = G::H * W * G::PS;
  extern __shared__ __attribute__((aligned(16))) bf16 lds_stb[];  // [IPW][dz (haloed) | dy]
  auto dzb = [&](int im) { return lds_stb + im * (G::IMGE + DYE); };
  auto dyb = [&](int im) { return lds_stb + im * (G::IMGE + DYE) + G::IMGE; };
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, lx = lane & 15;
  const int ot = wave % OT, rw = wave / OT;
  const float hg = h * two_gamma;
  for (int i = tid; i < IPW * (G::IMGE + DYE) / 8; i += G::NTH) ((uint4*)lds_stb)[i] = make_uint4(0u, 0u, 0u, 0u);
  for (int n0 = IPW * blockIdx.x; n0 < N; n0 += IPW * gridDim.x) {
    const int nimg = min(IPW, N - n0);  // (uniform)
    st_barrier();  // (the previous images' dx read out)
    for (int im = 0; im < nimg; ++im) {
      const long ib = (long)(n0 + im) * G::H * W * C;
      bf16* dst = dyb(im);
      st_fetch_image<G::NCH, G::NTH, uint4>(dyL + ib, tid, [&](int i, const uint4& v) {
        *(uint4*)(dst + (i / G::C8) * G::PS + 8 * (i % G::C8)) = v;
      });
    }
    for (int l = L - 1; l >= 0; --l) {
      bf16x8 A[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        A[ks] = *(const bf16x8*)(wpack + (long)l * w_stride + (((long)ot * KS + ks) * 64 + lane) * 8);
      // layer l's relu bits, loaded before the barrier (a byte load per chunk inside the loop below
      // waited for each in turn)
      const uint8_t* ml = masks + (long)l * mask_stride;
      constexpr int NPT = (G::NCH + G::NTH - 1) / G::NTH;
      unsigned mb[IPW][NPT];
#pragma unroll
      for (int im = 0; im < IPW; ++im)
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
          const int i = tid + k * G::NTH;
          mb[im][k] = (im < nimg && i < G::NCH) ? ml[((long)(n0 + im) * G::H * W * C + 8L * i) >> 3] : 0u;
        }
      st_barrier();  // dy of layer l complete (loaded, or the previous layer's dx); dz free
      for (int im = 0; im < nimg; ++im) {
        const long ib = (long)(n0 + im) * G::H * W * C;
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
          const int i = tid + k * G::NTH;
          if (i >= G::NCH) break;
          const int px = i / G::C8, c8 = i % G::C8;
          const uint4 v = *(const uint4*)(dyb(im) + px * G::PS + 8 * c8);
          *(uint4*)(dys + (long)l * d_stride + ib + 8L * i) = v;  // the gradient entering layer l (its wgrad's dy)
          *(uint4*)(dzb(im) + st_off<C, W>(px / W, px % W) + 8 * c8) = mask8_bf16(v, mb[im][k]);
        }
      }
      st_barrier();  // dz complete
      auto epi = [&](int im, int p, const f32x4& acc) {
        const int r = p / W, px = p % W;
        const int cz = st_off<C, W>(r, px) + 16 * ot + 4 * g, cy = p * G::PS + 16 * ot + 4 * g;
        const uint2 zw = *(const uint2*)(dzb(im) + cz), dw = *(const uint2*)(dyb(im) + cy);
        const float z4[4] = {__uint_as_float(zw.x << 16), __uint_as_float(zw.x & 0xffff0000u),
                             __uint_as_float(zw.y << 16), __uint_as_float(zw.y & 0xffff0000u)};
        const float d4[4] = {__uint_as_float(dw.x << 16), __uint_as_float(dw.x & 0xffff0000u),
                             __uint_as_float(dw.y << 16), __uint_as_float(dw.y & 0xffff0000u)};
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaf(hg, z4[e], fmaf(-h, acc[e], d4[e]));
        *(uint2*)(dyb(im) + cy) = make_uint2(pk_bf16_rn(v[0], v[1]), pk_bf16_rn(v[2], v[3]));  // (own pixel, own channels)
      };
#pragma unroll 1
      for (int j = 0; j < G::T / G::WPT; j += TP) {
        int pc[2], rc[2], xc[2];
        const bf16* bc[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          pc[c] = 16 * (rw + (j + c % TP) * G::WPT) + lx;
          rc[c] = pc[c] / W;
          xc[c] = pc[c] % W;
          bc[c] = dzb(c / TP);
        }
        f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const int kap = 32 * ks + 8 * g;
          const int t = min(kap / C, 8), i0c = kap - (kap / C) * C;
          uint4 b[2];
#pragma unroll
          for (int c = 0; c < 2; ++c)
            b[c] = *(const uint4*)(bc[c] + ((rc[c] + t / 3) * TW + xc[c] + t % 3) * G::PS + i0c);
#pragma unroll
          for (int c = 0; c < 2; ++c)
            acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[ks], __builtin_bit_cast(bf16x8, b[c]), acc[c], 0, 0, 0);
        }
        mfma_bf16_settle();
#pragma unroll
        for (int c = 0; c < 2; ++c)
          if (c / TP < nimg) epi(c / TP, pc[c], acc[c]);
      }
    }
    st_barrier();  // dx_0 complete
    for (int im = 0; im < nimg; ++im) {
      const long ib = (long)(n0 + im) * G::H * W * C;
      for (int i = tid; i < G::NCH; i += G::NTH)
        *(uint4*)(dx0 + ib + 8L * i) = *(const uint4*)(dyb(im) + (i / G::C8) * G::PS + 8 * (i % G::C8));
    }
  }
}

// ---------------------------------------------------------------------------
// The fp32 image-resident stages (k_stagef32 / k_stageb32: the reference's
// precision, v_mfma_f32_16x16x4_f32): the same structure as k_stagef /
// k_stageb with fp32 image tiles (pixel stride C + 4 floats, dynamic LDS) and
// the fp32 block's conventions: W in HWIO fp32, A = W^T fragments of the
// wave's o-tile in registers (k_conv32's), dz = h dy [relu bit] staged in
// fp32, dx = dy - conv(dz) + 2 gamma dz.
// ---------------------------------------------------------------------------
template <int C, int W_>
struct StImg32 {
  // NW waves per image: the fp32 MFMA is 4x the bf16's cycles per FLOP, and at the reference's batch
  // sizes (128) one 4-wave workgroup per image would leave half the SIMDs idle
  static constexpr int NW = 4, NTH = 64 * NW;
  static constexpr int W = W_, H = W_, TW = W + 2, OT = C / 16, OQ = C / 16, WPT = NW / OT, PS = C + 4;
  static constexpr int T = H * W / 16, IMGF = (H + 2) * TW * PS, NCH = H * W * C / 4;
  static_assert((W == 16 && C == 32) || (W == 8 && C == 64), "fp32 image-resident stage: 16 x 16 x 32 or 8 x 8 x 64");
};

template <int C, int W>
__device__ __forceinline__ int st32_off(int r, int c) {
  return ((r + 1) * StImg32<C, W>::TW + c + 1) * StImg32<C, W>::PS;
}

template <int C, int W>
__global__ __launch_bounds__((StImg32<C, W>::NTH)) void k_stagef32(const float* __restrict__ x0, float* __restrict__ ys, long y_stride,
                                                  uint8_t* __restrict__ masks, long mask_stride,
                                                  const float* __restrict__ w, long w_stride,
                                                  const float* __restrict__ bias, long bias_stride, float h, int N,
                                                  int L) {
  using G = StImg32<C, W>;
  constexpr int TW = G::TW, OQ = G::OQ, OT = G::OT, PS = G::PS;
  extern __shared__ __attribute__((aligned(16))) float lds_sf[];
  float* img0 = lds_sf;
  float* img1 = lds_sf + G::IMGF;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, lx = lane & 15;
  const int ot = wave % OT, rw = wave / OT;
  for (int i = tid; i < 2 * G::IMGF / 4; i += G::NTH) ((f32x4*)lds_sf)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  for (int n = blockIdx.x; n < N; n += gridDim.x) {
    const long ib = (long)n * G::H * W * C;
    st_fetch_image<G::NCH, G::NTH, f32x4>(x0 + ib, tid, [&](int i, const f32x4& v) {
      const int px = i / (C / 4), c4 = i % (C / 4);
      *(f32x4*)(img0 + st32_off<C, W>(px / W, px % W) + 4 * c4) = v;
    });
    __syncthreads();
    for (int l = 0; l < L; ++l) {
      const float* cur = (l & 1) ? img1 : img0;
      float* nxt = (l & 1) ? img0 : img1;
      const float* wl = w + (long)l * w_stride;
      float A[9][OQ][4];
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int q = 0; q < OQ; ++q)
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) A[t][q][s4] = wl[((long)t * C + 16 * q + 4 * g + s4) * C + 16 * ot + lx];
      const f32x4 bz = *(const f32x4*)(bias + (long)l * bias_stride + 16 * ot + 4 * g);
      float* yl = ys + (long)l * y_stride + ib;
      uint8_t* ml = masks + (long)l * mask_stride;
      auto epi = [&](int p, const f32x4& acc) {
        const int r = p / W, px = p % W;
        const int co = st32_off<C, W>(r, px) + 16 * ot + 4 * g;
        const f32x4 ctr = *(const f32x4*)(cur + co);
        f32x4 v;
        unsigned nib = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          nib |= (acc[e] > 0.f ? 1u : 0u) << e;
          v[e] = ctr[e] + h * fmaxf(acc[e], 0.f);
        }
        *(f32x4*)(nxt + co) = v;
        *(f32x4*)(yl + (long)p * C + 16 * ot + 4 * g) = v;
        const long pix = (long)n * G::H * W + p;
        unsigned m = nib << (4 * g);
        m |= (unsigned)__shfl_xor((int)m, 16, 64);
        m |= (unsigned)__shfl_xor((int)m, 32, 64);
        if (g == 0) *(uint16_t*)(ml + (pix * C + 16 * ot) / 8) = (uint16_t)m;
      };
#pragma unroll 1
      for (int j = 0; j < G::T / G::WPT; j += 2) {
        const int p0 = 16 * (rw + j * G::WPT) + lx, p1 = 16 * (rw + (j + 1) * G::WPT) + lx;
        const int r0 = p0 / W, x0p = p0 % W, r1 = p1 / W, x1p = p1 % W;
        f32x4 acc0 = bz, acc1 = bz;
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
          for (int q = 0; q < OQ; ++q) {
            const f32x4 b0 = *(const f32x4*)(cur + ((r0 + t / 3) * TW + x0p + t % 3) * PS + 16 * q + 4 * g);
            const f32x4 b1 = *(const f32x4*)(cur + ((r1 + t / 3) * TW + x1p + t % 3) * PS + 16 * q + 4 * g);
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
              acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(A[t][q][s4], b0[s4], acc0, 0, 0, 0);
              acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(A[t][q][s4], b1[s4], acc1, 0, 0, 0);
            }
          }
        mfma_f32_settle();
        epi(p0, acc0);
        epi(p1, acc1);
      }
      st_barrier();  // layer l's outputs complete in nxt; cur free
    }
  }
}

template <int C, int W>
__global__ __launch_bounds__((StImg32<C, W>::NTH)) void k_stageb32(const float* __restrict__ dyL, float* __restrict__ dys, long d_stride,
                                                  float* __restrict__ dx0, const uint8_t* __restrict__ masks,
                                                  long mask_stride, const float* __restrict__ w, long w_stride,
                                                  float h, float two_gamma, int N, int L) {
  using G = StImg32<C, W>;
  constexpr int TW = G::TW, OQ = G::OQ, OT = G::OT, PS = G::PS;
  extern __shared__ __attribute__((aligned(16))) float lds_sb[];
  float* dzt = lds_sb;              // dz = h dy [relu bit], zero halo
  float* dyt = lds_sb + G::IMGF;    // dy (becomes dx), pixel stride PS
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, lx = lane & 15;
  const int ot = wave % OT, rw = wave / OT;
  for (int i = tid; i < G::IMGF / 4; i += G::NTH) ((f32x4*)dzt)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int n = blockIdx.x; n < N; n += gridDim.x) {
    const long ib = (long)n * G::H * W * C;
    st_fetch_image<G::NCH, G::NTH, f32x4>(dyL + ib, tid, [&](int i, const f32x4& v) {
      *(f32x4*)(dyt + (i / (C / 4)) * PS + 4 * (i % (C / 4))) = v;
    });
    for (int l = L - 1; l >= 0; --l) {
      // layer l's relu bytes, loaded before the barrier (a byte load per chunk inside the loop below
      // waited for each in turn)
      const uint8_t* ml = masks + (long)l * mask_stride;
      constexpr int NPT = (G::NCH + G::NTH - 1) / G::NTH;
      unsigned mb[NPT];
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        const int i = tid + k * G::NTH;
        mb[k] = i < G::NCH ? ml[(ib + 4L * i) >> 3] : 0u;
      }
      st_barrier();  // dy of layer l complete; dz free
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        const int i = tid + k * G::NTH;
        if (i >= G::NCH) break;
        const int px = i / (C / 4), c4 = i % (C / 4);
        const f32x4 v = *(const f32x4*)(dyt + px * PS + 4 * c4);
        *(f32x4*)(dys + (long)l * d_stride + ib + 4L * i) = v;  // the gradient entering layer l (its wgrad's dy)
        const unsigned nib = mb[k] >> ((ib + 4L * i) & 7);  // (masked_dz4's bits: pixel * C + channel)
        f32x4 z;
#pragma unroll
        for (int j = 0; j < 4; ++j) z[j] = ((nib >> j) & 1u) ? h * v[j] : 0.f;
        *(f32x4*)(dzt + st32_off<C, W>(px / W, px % W) + 4 * c4) = z;
      }
      const float* wl = w + (long)l * w_stride;
      float A[9][OQ][4];
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int q = 0; q < OQ; ++q)
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) A[t][q][s4] = wl[((long)t * C + 16 * q + 4 * g + s4) * C + 16 * ot + lx];
      st_barrier();  // dz complete
      auto epi = [&](int p, const f32x4& acc) {
        const int r = p / W, px = p % W;
        const int cz = st32_off<C, W>(r, px) + 16 * ot + 4 * g, cy = p * PS + 16 * ot + 4 * g;
        const f32x4 z4 = *(const f32x4*)(dzt + cz), d4 = *(const f32x4*)(dyt + cy);
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = d4[e] - acc[e] + two_gamma * z4[e];
        *(f32x4*)(dyt + cy) = v;  // (own pixel, own channels)
      };
#pragma unroll 1
      for (int j = 0; j < G::T / G::WPT; j += 2) {
        const int p0 = 16 * (rw + j * G::WPT) + lx, p1 = 16 * (rw + (j + 1) * G::WPT) + lx;
        const int r0 = p0 / W, x0p = p0 % W, r1 = p1 / W, x1p = p1 % W;
        f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
          for (int q = 0; q < OQ; ++q) {
            const f32x4 b0 = *(const f32x4*)(dzt + ((r0 + t / 3) * TW + x0p + t % 3) * PS + 16 * q + 4 * g);
            const f32x4 b1 = *(const f32x4*)(dzt + ((r1 + t / 3) * TW + x1p + t % 3) * PS + 16 * q + 4 * g);
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
              acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(A[t][q][s4], b0[s4], acc0, 0, 0, 0);
              acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(A[t][q][s4], b1[s4], acc1, 0, 0, 0);
            }
          }
        mfma_f32_settle();
        epi(p0, acc0);
        epi(p1, acc1);
      }
    }
    st_barrier();  // dx_0 complete
    for (int i = tid; i < G::NCH; i += G::NTH)
      *(f32x4*)(dx0 + ib + 4L * i) = *(const f32x4*)(dyt + (i / (C / 4)) * PS + 4 * (i % (C / 4)));
    st_barrier();  // (dyt reused by the next image)
  }
}

bool stage_img32_supported(int H, int W, int C) { return H == W && ((W == 16 && C == 32) || (W == 8 && C == 64)); }

int stage_img32_forward(const float* x0, float* ys, long y_stride, uint8_t* masks, long mask_stride, const float* w,
                        long w_stride, const float* bias, long bias_stride, float h, int N, int H, int W, int C, int L,
                        hipStream_t s) {
  if (!stage_img32_supported(H, W, C)) return fail(ASR_E_UNSUPPORTED, "fp32 image-resident stage: H=%d W=%d C=%d", H, W, C);
  const unsigned grid = (unsigned)std::max(1, N);
#define ASR_SF32(CC, WW)                                                                                             \
  if (C == CC && W == WW) {                                                                                          \
    using GG = StImg32<CC, WW>;                                                                                      \
    const size_t lds = (size_t)2 * GG::IMGF * 4;                                                                     \
    hipLaunchKernelGGL((k_stagef32<CC, WW>), dim3(grid), dim3(GG::NTH), lds, s, x0, ys, y_stride, masks, mask_stride, w, \
                       w_stride, bias, bias_stride, h, N, L);                                                        \
    ASR_LAUNCH_CHECK("k_stagef32");                                                                                  \
    return ASR_OK;                                                                                                   \
  }
  ASR_SF32(32, 16) ASR_SF32(64, 8)
#undef ASR_SF32
  return fail(ASR_E_UNSUPPORTED, "fp32 image-resident stage: C=%d W=%d", C, W);
}

int stage_img32_backward(const float* dyL, float* dys, long d_stride, float* dx0, const uint8_t* masks,
                         long mask_stride, const float* w, long w_stride, float h, float two_gamma, int N, int H, int W,
                         int C, int L, hipStream_t s) {
  if (!stage_img32_supported(H, W, C)) return fail(ASR_E_UNSUPPORTED, "fp32 image-resident stage: H=%d W=%d C=%d", H, W, C);
  const unsigned grid = (unsigned)std::max(1, N);
#define ASR_SB32(CC, WW)                                                                                            \
  if (C == CC && W == WW) {                                                                                         \
    using GG = StImg32<CC, WW>;                                                                                     \
    const size_t lds = (size_t)(GG::IMGF + GG::H * WW * GG::PS) * 4;                                                \
    hipLaunchKernelGGL((k_stageb32<CC, WW>), dim3(grid), dim3(GG::NTH), lds, s, dyL, dys, d_stride, dx0, masks,     \
                       mask_stride, w, w_stride, h, two_gamma, N, L);                                               \
    ASR_LAUNCH_CHECK("k_stageb32");                                                                                 \
    return ASR_OK;                                                                                                  \
  }
  ASR_SB32(32, 16) ASR_SB32(64, 8)
#undef ASR_SB32
  return fail(ASR_E_UNSUPPORTED, "fp32 image-resident stage: C=%d W=%d", C, W);
}

// every layer's fp32 weight-gradient slabs in one launch (k_wgrad32, blockIdx.y = layer)
int wgrad32_layers(const float* x0, long x_stride, const float* dys, long d_stride, const uint8_t* masks,
                   long mask_stride, float h, int N, int H, int W, int C, int L, float* slabs, long slab_stride,
                   int* nslabs, hipStream_t s) {
#define ASR_W32L(CC, WW)                                                                                     \
  if (C == CC && W == WW)                                                                                    \
    return launch_wgrad32<CC, WW>(x0, dys, N, H, slabs, nslabs, s, masks, h, L, x_stride, d_stride, mask_stride, \
                                  slab_stride);
  ASR_W32L(32, 16) ASR_W32L(64, 8) ASR_W32L(16, 32) ASR_W32L(32, 32) ASR_W32L(64, 16)
#undef ASR_W32L
  return fail(ASR_E_UNSUPPORTED, "fp32 weight gradient (layers): C=%d W=%d", C, W);
}

bool stage_img_supported(int H, int W, int C) {
  return H == W && ((W == 16 && C == 32) || (W == 8 && C == 64) || (W == 8 && C == 32));
}

// the image-resident stage forward: x0 [N][H][W][C] -> ys (L layers at y_stride), masks (L at mask_stride)
int stage_img_forward(const void* x0, void* ys, long y_stride, uint8_t* masks, long mask_stride, const void* w,
                      long w_stride, const float* bias, long bias_stride, float h, int N, int H, int W, int C, int L,
                      hipStream_t s) {
  if (!stage_img_supported(H, W, C)) return fail(ASR_E_UNSUPPORTED, "image-resident stage: H=%d W=%d C=%d", H, W, C);
  const unsigned grid = (unsigned)std::max(1, (N + kStIpw - 1) / kStIpw);
#define ASR_SF(CC, WW)                                                                                        \
  if (C == CC && W == WW) {                                                                                   \
    const size_t lds = (size_t)kStIpw * 2 * StImg<CC, WW>::IMGE * 2;                                      \
    hipLaunchKernelGGL((k_stagef<CC, WW>), dim3(grid), dim3(StImg<CC, WW>::NTH), lds, s, (const bf16*)x0, (bf16*)ys, \
                       y_stride,                                                                              \
                       masks, mask_stride, (const bf16*)w, w_stride, bias, bias_stride, h, N, L);             \
    ASR_LAUNCH_CHECK("k_stagef");                                                                             \
    return ASR_OK;                                                                                            \
  }
  ASR_SF(32, 16) ASR_SF(64, 8)
  ASR_SF(32, 8)
#undef ASR_SF
  return fail(ASR_E_UNSUPPORTED, "image-resident stage: C=%d W=%d", C, W);
}

// its backward (input gradient): dyL -> dx0; dys: the gradient entering each layer 0 .. L-1 (d_stride apart)
int stage_img_backward(const void* dyL, void* dys, long d_stride, void* dx0, const uint8_t* masks, long mask_stride,
                       const void* w, long w_stride, float h, float two_gamma, int N, int H, int W, int C, int L,
                       hipStream_t s) {
  if (!stage_img_supported(H, W, C)) return fail(ASR_E_UNSUPPORTED, "image-resident stage: H=%d W=%d C=%d", H, W, C);
  const unsigned grid = (unsigned)std::max(1, (N + kStIpw - 1) / kStIpw);
#define ASR_SB(CC, WW)                                                                                           \
  if (C == CC && W == WW) {                                                                                      \
    using GG = StImg<CC, WW>;                                                                                    \
    const size_t lds = (size_t)kStIpw * (GG::IMGE + GG::H * WW * GG::PS) * 2;                                \
    hipLaunchKernelGGL((k_stageb<CC, WW>), dim3(grid), dim3(GG::NTH), lds, s, (const bf16*)dyL, (bf16*)dys, d_stride, \
                       (bf16*)dx0, masks, mask_stride, (const bf16*)w, w_stride, h, two_gamma, N, L);             \
    ASR_LAUNCH_CHECK("k_stageb");                                                                                \
    return ASR_OK;                                                                                               \
  }
  ASR_SB(32, 16) ASR_SB(64, 8)
  ASR_SB(32, 8)
#undef ASR_SB
  return fail(ASR_E_UNSUPPORTED, "image-resident stage: C=%d W=%d", C, W);
}

// the weight-gradient slabs of L layers in one launch (k_wgradb, blockIdx.y = layer): layer l reads
// x0 + l x_stride, dys + l d_stride, masks + l mask_stride and writes slabs + l slab_stride
int wgradb_layers(const void* x0, long x_stride, const void* dys, long d_stride, const uint8_t* masks,
                  long mask_stride, float h, int N, int H, int W, int C, int L, float* slabs, long slab_stride,
                  int* nslabs, hipStream_t s) {
#define ASR_WL(CC, WW)                                                                                              \
  if (C == CC && W == WW)                                                                                           \
    return launch_wgradb<CC, WW>((const bf16*)x0, (const bf16*)dys, masks, N, H, h, slabs, nslabs, s, L, x_stride, \
                                 d_stride, mask_stride, slab_stride);
  ASR_WL(16, 32) ASR_WL(16, 16) ASR_WL(16, 8) ASR_WL(32, 32) ASR_WL(32, 16) ASR_WL(32, 8) ASR_WL(64, 32)
  ASR_WL(64, 16) ASR_WL(64, 8)
#undef ASR_WL
  return fail(ASR_E_UNSUPPORTED, "bf16 weight gradient: C=%d W=%d", C, W);
}

// elementwise bf16 <-> fp32 (the multi-stage bf16 net's transitions run in fp32)
__global__ void k_bf16_to_f32(const bf16* __restrict__ a, float* __restrict__ b, long n8) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    const uint4 u = ((const uint4*)a)[i];
    const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      ((float2*)b)[4 * i + k] = make_float2(__uint_as_float(w[k] << 16), __uint_as_float(w[k] & 0xffff0000u));
  }
}
__global__ void k_f32_to_bf16(const float* __restrict__ a, bf16* __restrict__ b, long n8) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    const float4 p = ((const float4*)a)[2 * i], q = ((const float4*)a)[2 * i + 1];
    ((uint4*)b)[i] = make_uint4(pk_bf16_rn(p.x, p.y), pk_bf16_rn(p.z, p.w), pk_bf16_rn(q.x, q.y), pk_bf16_rn(q.z, q.w));
  }
}
int convert_bf16_f32(const void* src, void* dst, long n, int to_f32, hipStream_t s) {
  if (n % 8) return fail(ASR_E_ARG, "bf16 <-> fp32: element count %ld not a multiple of 8", n);
  const long n8 = n / 8;
  const unsigned grid = (unsigned)std::max<long>(1, std::min<long>((n8 + 255) / 256, 8192));
  if (to_f32)
    hipLaunchKernelGGL(k_bf16_to_f32, dim3(grid), dim3(256), 0, s, (const bf16*)src, (float*)dst, n8);
  else
    hipLaunchKernelGGL(k_f32_to_bf16, dim3(grid), dim3(256), 0, s, (const float*)src, (bf16*)dst, n8);
  ASR_LAUNCH_CHECK("k_bf16_f32");
  return ASR_OK;
}

}  // namespace asr
