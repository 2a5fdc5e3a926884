// Multi-stage single-block ResNet (ABI 7, include/asr.h "Multi-stage"): the
// stage transition single_layer_conv_block (models/tfkeras_resnets.py:204-269)
// as fp32 kernels, and the executor of get_single_block_resnet_build_function
// with num_stages > 2 (tfkeras_resnets.py:547-597, e.g. the He-style ResNet-32:
// [10, 10, 10] blocks at 32^2 x 16, 16^2 x 32, 8^2 x 64).
//
// The identity blocks of every stage run the fp32 block kernels of the
// single-stage executor (asr_conv_forward / asr_conv_backward: fp32 MFMA for
// C in {16, 32, 64} at W in {32, 16, 8}, the fp32 VALU kernel otherwise); the
// stem and head are the single-stage executor's kernels.
//
// Transition, for output pixel p = (n, yo, xo) and channel o (stride S, TF
// 'same' padding for the 3x3: pad_top = ((Ho-1)S + 3 - H) / 2, the remainder
// at the bottom / right; the 1x1 is 'valid', i.e. it reads input (S yo, S xo)):
//     z  = b2[o] + sum_{ky,kx,i} x[S yo + ky - pt][S xo + kx - pl][i] K2[ky][kx][i][o]
//     y  = relu(z) + b1[o] + sum_i x[S yo][S xo][i] K1[i][o]
// Backward (dz = dy [z > 0]):
//     dx[gy][gx][i] = sum_{ky,kx: gy + pt - ky = S yo, gx + pl - kx = S xo} sum_o dz[yo][xo][o] K2[ky][kx][i][o]
//                   + [S | gy, S | gx] sum_o dy[gy/S][gx/S][o] K1[i][o]
//     dK2[ky][kx][i][o] = sum_p x[S yo + ky - pt][S xo + kx - pl][i] dz[p][o],  db2 = sum_p dz
//     dK1[i][o]         = sum_p x[S yo][S xo][i] dy[p][o],                     db1 = sum_p dy
// These convolutions carry ~2 % of a ResNet-32 step's FLOPs (two transitions
// against 28 identity blocks).  With Ci, Co multiples of 16 they run on the
// fp32 matrix cores (k_trans_*_mfma, one wave per 16 x 16 output tile,
// operands from global memory); other shapes on the VALU: one lane per
// (pixel, 4 output channels) in the forward, per (input pixel, channel) in
// dgrad, per weight element over a chunk of output rows in wgrad.  Weight
// gradient partials per chunk are reduced by one more launch.
#include <algorithm>
#include <vector>

#include "asr_common.h"

namespace asr {
// asr_theta.hip
long theta_count(int C, int kind, int antisymmetric);
int param_map(int C, int kind, int antisymmetric, int32_t* w_src, int32_t* theta_dst);
int param_is_antisymmetric(int kind, int antisymmetric);
int param_map_transpose(int C, const int32_t* w_src, int32_t* w_bwd);
int reduce_and_project(const float* slabs, int P, long E, int Cb, const int32_t* theta_dst, long n_theta,
                       float* dtheta, float* dbias, float* dw_out, float* ws, hipStream_t s);
size_t reduce_ws_bytes(int P, long ES);
int reduce_groups(int P);
int f32_block_slab_rows(int N, int H, int W, int C);
int project_layers(float* grp, long grp_stride, int G, long E, int Cb, const int32_t* theta_dst, long n_theta,
                   int L, float* out, long out_stride, hipStream_t s);
int reduce_slab_layers(const float* slabs, long slab_stride, int P, long ES, float* grp, long grp_stride, int L,
                       hipStream_t s);
// asr_conv_f32.hip: the bf16 blocks at any stage width, bf16 <-> fp32
bool convb_supported(int W, int C);
int convb_forward(const void* x, void* y, uint8_t* mask, const void* w, const float* bias, float h, int N, int H, int W,
                  int C, hipStream_t s, bool conv_only = false);
int convb_backward(const void* dy, const uint8_t* mask, const void* x, const void* w, float h, float two_gamma, int N,
                   int H, int W, int C, void* dx, bool need_w, float* slabs, int* nslabs, hipStream_t s,
                   bool conv_only = false);
int convert_bf16_f32(const void* src, void* dst, long n, int to_f32, hipStream_t s);
bool stage_img_supported(int H, int W, int C);
int stage_img_forward(const void* x0, void* ys, long y_stride, uint8_t* masks, long mask_stride, const void* w,
                      long w_stride, const float* bias, long bias_stride, float h, int N, int H, int W, int C, int L,
                      hipStream_t s);
int stage_img_backward(const void* dyL, void* dys, long d_stride, void* dx0, const uint8_t* masks, long mask_stride,
                       const void* w, long w_stride, float h, float two_gamma, int N, int H, int W, int C, int L,
                       hipStream_t s);
bool stage_img32_supported(int H, int W, int C);
int stage_img32_forward(const float* x0, float* ys, long y_stride, uint8_t* masks, long mask_stride, const float* w,
                        long w_stride, const float* bias, long bias_stride, float h, int N, int H, int W, int C, int L,
                        hipStream_t s);
int stage_img32_backward(const float* dyL, float* dys, long d_stride, float* dx0, const uint8_t* masks,
                         long mask_stride, const float* w, long w_stride, float h, float two_gamma, int N, int H, int W,
                         int C, int L, hipStream_t s);
int wgrad32_layers(const float* x0, long x_stride, const float* dys, long d_stride, const uint8_t* masks,
                   long mask_stride, float h, int N, int H, int W, int C, int L, float* slabs, long slab_stride,
                   int* nslabs, hipStream_t s);
int wgradb_layers(const void* x0, long x_stride, const void* dys, long d_stride, const uint8_t* masks,
                  long mask_stride, float h, int N, int H, int W, int C, int L, float* slabs, long slab_stride,
                  int* nslabs, hipStream_t s);
// asr_deep16.hip: the C = 16, 32 x 32 bf16 stage as one fused forward / backward launch
bool deep16_supported(int H, int W, int C);
int deep16_forward(const void* x0, void* y0, long y_stride, uint8_t* mask0, long mask_stride, const void* wpack,
                   const float* bias, long bias_stride, float h, int N, int L, bool store_all, hipStream_t s);
size_t deep16_slab_bytes(int N, int L);
int deep16_backward(void* dbufA, void* dbufB, const void* xs, long x_stride, const uint8_t* masks, long mask_stride,
                    const void* wpack, float h, float two_gamma, int N, int L, float* slabs, int* slab_rows,
                    int* dx0_in_b, hipStream_t s);
// asr_theta.hip
int reduce_slabs_to_groups(const float* slabs, int P, long ES, float* grp, hipStream_t s);
// asr_api.hip
int conv_backward_keep_slabs(const void* dy, const void* x, const uint8_t* mask, const void* w, float h, float gamma,
                             int N, int H, int W, int C, void* dx, void* ws, float* slabs, int* nsl, hipStream_t s);
// asr_stem_head.hip
bool stem_supported(int Cin, int H, int W, int C);
int stem_forward(const void* img, int input_u8, const float* w1, const float* b1, int N, int H, int W, int Cin, int C,
                 float mean, float inv_std, int use_norm, void* out, int out_bf16, hipStream_t s);
int stem_wgrad_mfma(const void* img, int input_u8, const void* dz1, int N, int H, int W, int Cin, int C, float mean,
                    float inv_std, int use_norm, float* slabs, int* nslabs, hipStream_t s);
bool stem_wgrad_mfma_supported(int Cin, int H, int W, int C);
int relu_grad_bf16(void* d, const void* x, long n, hipStream_t s);
int stem_wgrad(const void* img, int input_u8, const void* dx1, const void* x1, int act_bf16, int N, int H, int W,
               int Cin, int C, float mean, float inv_std, int use_norm, float* slabs, int* nslabs, hipStream_t s);
int head(const void* xL, int act_bf16, const float* fck, const float* fcb, const float* targets, int N, int HW, int C,
         int K, float* probs, float* loss_per, float* dlogits, float* gap, void* dxL, hipStream_t s,
         void* growL = nullptr);
int head_param_grads(const float* gap, const float* dlogits, int N, int C, int K, float* dfck, float* dfcb,
                     const float* loss_per, float* loss_out, hipStream_t s);

namespace {

constexpr int kTK = 3;              // the transition's kxk (the builder's kernel_size; 3 in every reference config)
constexpr int kMaxTransChunks = 256;  // wgrad row chunks
constexpr int kMaxStemSlabs = 512;    // asr_stem_head.hip stem_grid bound

struct TGeom {
  int Ho, Wo, pt, pl;
};
TGeom tgeom(int H, int W, int S) {
  TGeom g;
  g.Ho = (H + S - 1) / S;
  g.Wo = (W + S - 1) / S;
  g.pt = std::max((g.Ho - 1) * S + kTK - H, 0) / 2;
  g.pl = std::max((g.Wo - 1) * S + kTK - W, 0) / 2;
  return g;
}
long trans_param_floats(int Ci, int Co) { return (long)kTK * kTK * Ci * Co + Co + (long)Ci * Co + Co; }

// one wave = (n, yo, 16-pixel tile, 16-channel tile); lane (lx, g): pixel 16 pt + lx, channels o0 .. o0 + 3
__global__ __launch_bounds__(256) void k_trans_fwd(const float* __restrict__ x, float* __restrict__ y,
                                                   uint8_t* __restrict__ mask, const float* __restrict__ k2,
                                                   const float* __restrict__ b2, const float* __restrict__ k1,
                                                   const float* __restrict__ b1, int N, int H, int W, int Ci, int Co,
                                                   int S, int Ho, int Wo, int pt, int pl) {
  const int PT = (Wo + 15) / 16, OT = (Co + 15) / 16;
  const long tasks = (long)N * Ho * PT * OT;
  const long task = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (task >= tasks) return;
  const int lane = threadIdx.x & 63, g = lane >> 4, lx = lane & 15;
  const int ot = (int)(task % OT);
  long rest = task / OT;
  const int ptile = (int)(rest % PT);
  rest /= PT;
  const int yo = (int)(rest % Ho);
  const int n = (int)(rest / Ho);
  const int xo = 16 * ptile + lx, o0 = 16 * ot + 4 * g;
  if (xo >= Wo || o0 >= Co) return;
  const int no = min(4, Co - o0);
  float z[4] = {0.f, 0.f, 0.f, 0.f}, sc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int ky = 0; ky < kTK; ++ky) {
    const int gy = S * yo + ky - pt;
    if (gy < 0 || gy >= H) continue;
    for (int kx = 0; kx < kTK; ++kx) {
      const int gx = S * xo + kx - pl;
      if (gx < 0 || gx >= W) continue;
      const float* xp = x + (((long)n * H + gy) * W + gx) * Ci;
      const float* wp = k2 + (long)(ky * kTK + kx) * Ci * Co + o0;
      for (int i = 0; i < Ci; ++i) {
        const float xv = xp[i];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (e < no) z[e] = fmaf(xv, wp[(long)i * Co + e], z[e]);
      }
    }
  }
  {
    const float* xp = x + (((long)n * H + S * yo) * W + S * xo) * Ci;
    for (int i = 0; i < Ci; ++i) {
      const float xv = xp[i];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (e < no) sc[e] = fmaf(xv, k1[(long)i * Co + o0 + e], sc[e]);
    }
  }
  const long p = ((long)n * Ho + yo) * Wo + xo;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (e >= no) continue;
    const int o = o0 + e;
    const float zz = z[e] + b2[o];
    y[p * Co + o] = fmaxf(zz, 0.f) + (sc[e] + b1[o]);
    if (mask) mask[p * Co + o] = zz > 0.f ? 1 : 0;
  }
}

// one thread per (n, gy, gx, i)
__global__ __launch_bounds__(256) void k_trans_dgrad(const float* __restrict__ dy, const uint8_t* __restrict__ mask,
                                                     const float* __restrict__ k2, const float* __restrict__ k1,
                                                     float* __restrict__ dx, int N, int H, int W, int Ci, int Co,
                                                     int S, int Ho, int Wo, int pt, int pl) {
  const long total = (long)N * H * W * Ci;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int i = (int)(idx % Ci);
    long rest = idx / Ci;
    const int gx = (int)(rest % W);
    rest /= W;
    const int gy = (int)(rest % H);
    const int n = (int)(rest / H);
    float acc = 0.f;
    for (int ky = 0; ky < kTK; ++ky) {
      const int ty = gy + pt - ky;
      if (ty < 0 || ty % S) continue;
      const int yo = ty / S;
      if (yo >= Ho) continue;
      for (int kx = 0; kx < kTK; ++kx) {
        const int tx = gx + pl - kx;
        if (tx < 0 || tx % S) continue;
        const int xo = tx / S;
        if (xo >= Wo) continue;
        const long p = ((long)n * Ho + yo) * Wo + xo;
        const float* dp = dy + p * Co;
        const uint8_t* mp = mask + p * Co;
        const float* wp = k2 + ((long)(ky * kTK + kx) * Ci + i) * Co;
        for (int o = 0; o < Co; ++o)
          if (mp[o]) acc = fmaf(dp[o], wp[o], acc);
      }
    }
    if (gy % S == 0 && gx % S == 0 && gy / S < Ho && gx / S < Wo) {
      const float* dp = dy + (((long)n * Ho + gy / S) * Wo + gx / S) * Co;
      const float* wp = k1 + (long)i * Co;
      for (int o = 0; o < Co; ++o) acc = fmaf(dp[o], wp[o], acc);
    }
    dx[idx] = acc;
  }
}

// partial [dK2 | db2 | dK1 | db1] of one chunk of output rows (n, yo) per blockIdx.y
__global__ __launch_bounds__(256) void k_trans_wgrad(const float* __restrict__ dy, const uint8_t* __restrict__ mask,
                                                     const float* __restrict__ x, float* __restrict__ part, int N,
                                                     int H, int W, int Ci, int Co, int S, int Ho, int Wo, int pt,
                                                     int pl, int rows_per_chunk) {
  const long E2 = (long)kTK * kTK * Ci * Co, E1 = (long)Ci * Co, ET = E2 + Co + E1 + Co;
  const long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (e >= ET) return;
  // decode the element: which sum, which operands
  int kind, ky = 0, kx = 0, i = 0, o;
  if (e < E2) {
    kind = 0;
    o = (int)(e % Co);
    i = (int)((e / Co) % Ci);
    const int tap = (int)(e / ((long)Ci * Co));
    ky = tap / kTK;
    kx = tap % kTK;
  } else if (e < E2 + Co) {
    kind = 1;
    o = (int)(e - E2);
  } else if (e < E2 + Co + E1) {
    kind = 2;
    const long f = e - E2 - Co;
    o = (int)(f % Co);
    i = (int)(f / Co);
  } else {
    kind = 3;
    o = (int)(e - E2 - Co - E1);
  }
  const long R = (long)N * Ho;
  const long r0 = (long)blockIdx.y * rows_per_chunk, r1 = min(R, r0 + rows_per_chunk);
  float acc = 0.f;
  for (long rr = r0; rr < r1; ++rr) {
    const int yo = (int)(rr % Ho);
    const int n = (int)(rr / Ho);
    const float* dr = dy + rr * Wo * Co;
    const uint8_t* mr = mask + rr * Wo * Co;
    if (kind == 0) {
      const int gy = S * yo + ky - pt;
      if (gy < 0 || gy >= H) continue;
      const float* xr = x + ((long)n * H + gy) * W * Ci;
      for (int xo = 0; xo < Wo; ++xo) {
        const int gx = S * xo + kx - pl;
        if (gx < 0 || gx >= W) continue;
        if (mr[(long)xo * Co + o]) acc = fmaf(xr[(long)gx * Ci + i], dr[(long)xo * Co + o], acc);
      }
    } else if (kind == 1) {
      for (int xo = 0; xo < Wo; ++xo)
        if (mr[(long)xo * Co + o]) acc += dr[(long)xo * Co + o];
    } else if (kind == 2) {
      const float* xr = x + ((long)n * H + S * yo) * W * Ci;
      for (int xo = 0; xo < Wo; ++xo) acc = fmaf(xr[(long)S * xo * Ci + i], dr[(long)xo * Co + o], acc);
    } else {
      for (int xo = 0; xo < Wo; ++xo) acc += dr[(long)xo * Co + o];
    }
  }
  part[(long)blockIdx.y * ET + e] = acc;
}

// out[e] = sum_c part[c][e]: a workgroup = 64 elements x 4 chunk slices, 4 independent
// partial sums per thread (loads in flight), the slices combined through LDS in a fixed order
__global__ __launch_bounds__(256) void k_sum_chunks(const float* __restrict__ part, int chunks, long E,
                                                    float* __restrict__ out) {
  __shared__ float red[4][64];
  const int lx = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const long e = blockIdx.x * 64L + lx;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (e < E) {
    int c = sl;
#pragma unroll 4  // (unrolled, the later iterations' loads issue before the earlier adds: same sums)
    for (; c + 12 < chunks; c += 16) {
      a0 += part[(long)c * E + e];
      a1 += part[(long)(c + 4) * E + e];
      a2 += part[(long)(c + 8) * E + e];
      a3 += part[(long)(c + 12) * E + e];
    }
    for (; c < chunks; c += 4) a0 += part[(long)c * E + e];
  }
  red[sl][lx] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (sl == 0 && e < E) out[e] = (red[0][lx] + red[1][lx]) + (red[2][lx] + red[3][lx]);
}

// ---------------------------------------------------------------------------
// the same three convolutions on the fp32 matrix cores (v_mfma_f32_16x16x4_f32,
// fp32 products and accumulation) when Ci and Co are multiples of 16 (every
// transition of the reference's ResNets).  One wave per 16 x 16 output tile;
// operands straight from global memory (L1/L2-resident weights and rows).
// Lane (lx, g) of an MFMA step s over a 16-channel group q supplies reduction
// index 16q + 4g + s for both operands, so A / B are 16-B loads of 4
// consecutive channels; the accumulator lane (lx, g) holds rows 4g .. 4g+3 of
// column lx.
// ---------------------------------------------------------------------------
__device__ __forceinline__ f32x4 ld4(const float* p) { return *(const f32x4*)p; }
// 4 consecutive bf16 as fp32 (the bf16 nets' activations, exact)
__device__ __forceinline__ f32x4 ld4(const bf16* p) {
  const uint2 u = *(const uint2*)p;
  return f32x4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
               __uint_as_float(u.y & 0xffff0000u)};
}
__device__ __forceinline__ void st4(float* p, f32x4 v) { *(f32x4*)p = v; }
__device__ __forceinline__ void st4(bf16* p, f32x4 v) {
  *(uint2*)p = make_uint2(pk_bf16_rn(v[0], v[1]), pk_bf16_rn(v[2], v[3]));
}
__device__ __forceinline__ f32x4 mask4u(unsigned u) {
  return f32x4{(float)(u & 0xff), (float)((u >> 8) & 0xff), (float)((u >> 16) & 0xff), (float)(u >> 24)};
}
__device__ __forceinline__ f32x4 mask4(const uint8_t* m) { return mask4u(*(const unsigned*)m); }

// Stage TOTAL 16-B elements with NT threads into LDS, BS at a time: load(i, v, m) fills an
// element (v and m zero unless it loads), store(i, v, m) writes it.  All BS loads issue
// before the first store (a rolled load-then-store loop waits for each load in turn).
template <int TOTAL, int NT, typename LoadF, typename StoreF>
__device__ __forceinline__ void stage_batched(int tid, LoadF load, StoreF store) {
  constexpr int NI = (TOTAL + NT - 1) / NT, BS = 4;
#pragma unroll
  for (int k0 = 0; k0 < NI; k0 += BS) {
    f32x4 v[BS];
    unsigned m[BS];
#pragma unroll
    for (int k = 0; k < BS; ++k) {
      v[k] = f32x4{0.f, 0.f, 0.f, 0.f};
      m[k] = 0u;
      const int i = tid + (k0 + k) * NT;
      if (k0 + k < NI && i < TOTAL) load(i, v[k], m[k]);
    }
#pragma unroll
    for (int k = 0; k < BS; ++k) {
      const int i = tid + (k0 + k) * NT;
      if (k0 + k < NI && i < TOTAL) store(i, v[k], m[k]);
    }
  }
}

// forward: D[o][xo] over (tap, i) + the 1x1 shortcut; wave = (n, yo, 16 xo, 16 o)
__global__ __launch_bounds__(256) void k_trans_fwd_mfma(const float* __restrict__ x, float* __restrict__ y,
                                                        uint8_t* __restrict__ mask, const float* __restrict__ k2,
                                                        const float* __restrict__ b2, const float* __restrict__ k1,
                                                        const float* __restrict__ b1, int N, int H, int W, int Ci,
                                                        int Co, int S, int Ho, int Wo, int pt, int pl) {
  const int PT = (Wo + 15) / 16, OT = Co / 16;
  const long task = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (task >= (long)N * Ho * PT * OT) return;
  const int lane = threadIdx.x & 63, g = lane >> 4, lx = lane & 15;
  const int ot = (int)(task % OT);
  long rest = task / OT;
  const int ptile = (int)(rest % PT);
  rest /= PT;
  const int yo = (int)(rest % Ho), n = (int)(rest / Ho);
  const int xo = 16 * ptile + lx;  // the B column (pixel) of this lane
  const int o = 16 * ot + lx;      // the A row (output channel) of this lane
  f32x4 acc = {0.f, 0.f, 0.f, 0.f}, accs = {0.f, 0.f, 0.f, 0.f};
  for (int ky = 0; ky < kTK; ++ky) {
    const int gy = S * yo + ky - pt;
    if (gy < 0 || gy >= H) continue;  // (wave-uniform)
    for (int kx = 0; kx < kTK; ++kx) {
      const int gx = S * xo + kx - pl;
      const bool ok = xo < Wo && gx >= 0 && gx < W;
      const float* xp = x + (((long)n * H + gy) * W + (ok ? gx : 0)) * Ci + 4 * g;
      const float* wp = k2 + (long)(ky * kTK + kx) * Ci * Co + (long)(4 * g) * Co + o;
      for (int q = 0; q < Ci / 16; ++q) {
        const f32x4 bv = ok ? ld4(xp + 16 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wp[(long)(16 * q + s4) * Co], bv[s4], acc, 0, 0, 0);
      }
    }
  }
  {
    const bool ok = xo < Wo;
    const float* xp = x + (((long)n * H + S * yo) * W + (ok ? S * xo : 0)) * Ci + 4 * g;
    const float* wp = k1 + (long)(4 * g) * Co + o;
    for (int q = 0; q < Ci / 16; ++q) {
      const f32x4 bv = ok ? ld4(xp + 16 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
        accs = __builtin_amdgcn_mfma_f32_16x16x4f32(wp[(long)(16 * q + s4) * Co], bv[s4], accs, 0, 0, 0);
    }
  }
  if (xo >= Wo) return;
  const long p = ((long)n * Ho + yo) * Wo + xo;
  const int o0 = 16 * ot + 4 * g;  // this lane's 4 output channels (accumulator rows)
  const f32x4 bb2 = ld4(b2 + o0), bb1 = ld4(b1 + o0);
  f32x4 v;
  unsigned mb = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float z = acc[j] + bb2[j];
    v[j] = fmaxf(z, 0.f) + (accs[j] + bb1[j]);
    mb |= (z > 0.f ? 1u : 0u) << (8 * j);
  }
  *(f32x4*)(y + p * Co + o0) = v;
  if (mask) *(unsigned*)(mask + p * Co + o0) = mb;
}

// dgrad: D[i][gx] over (tap, o) of dz = dy [z > 0] + the shortcut's dy; wave = (n, gy, 16 gx, 16 i)
__global__ __launch_bounds__(256) void k_trans_dgrad_mfma(const float* __restrict__ dy, const uint8_t* __restrict__ mask,
                                                          const float* __restrict__ k2, const float* __restrict__ k1,
                                                          float* __restrict__ dx, int N, int H, int W, int Ci, int Co,
                                                          int S, int Ho, int Wo, int pt, int pl) {
  const int PT = (W + 15) / 16, IT = Ci / 16;
  const long task = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (task >= (long)N * H * PT * IT) return;
  const int lane = threadIdx.x & 63, g = lane >> 4, lx = lane & 15;
  const int it = (int)(task % IT);
  long rest = task / IT;
  const int ptile = (int)(rest % PT);
  rest /= PT;
  const int gy = (int)(rest % H), n = (int)(rest / H);
  const int gx = 16 * ptile + lx;  // B column (input pixel)
  const int i = 16 * it + lx;      // A row (input channel)
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int ky = 0; ky < kTK; ++ky) {
    const int ty = gy + pt - ky;
    if (ty < 0 || ty % S) continue;  // (wave-uniform)
    const int yo = ty / S;
    if (yo >= Ho) continue;
    for (int kx = 0; kx < kTK; ++kx) {
      const int tx = gx + pl - kx;
      const bool ok = gx < W && tx >= 0 && tx % S == 0 && tx / S < Wo;
      const long p = ((long)n * Ho + yo) * Wo + (ok ? tx / S : 0);
      const float* dp = dy + p * Co + 4 * g;
      const uint8_t* mp = mask + p * Co + 4 * g;
      const float* wp = k2 + ((long)(ky * kTK + kx) * Ci + i) * Co + 4 * g;
      for (int q = 0; q < Co / 16; ++q) {
        const f32x4 av = ld4(wp + 16 * q);
        const f32x4 bv = ok ? ld4(dp + 16 * q) * mask4(mp + 16 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s4], bv[s4], acc, 0, 0, 0);
      }
    }
  }
  if (gy % S == 0 && gy / S < Ho) {  // (wave-uniform)
    const bool ok = gx < W && gx % S == 0 && gx / S < Wo;
    const float* dp = dy + (((long)n * Ho + gy / S) * Wo + (ok ? gx / S : 0)) * Co + 4 * g;
    const float* wp = k1 + (long)i * Co + 4 * g;
    for (int q = 0; q < Co / 16; ++q) {
      const f32x4 av = ld4(wp + 16 * q);
      const f32x4 bv = ok ? ld4(dp + 16 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s4], bv[s4], acc, 0, 0, 0);
    }
  }
  if (gx < W) *(f32x4*)(dx + (((long)n * H + gy) * W + gx) * Ci + 16 * it + 4 * g) = acc;
}

// wgrad partials: wave = (chunk of output pixels, 16 i, 16 o); the 9 taps' D[i][o] = sum_p x_tap[p][i] dz[p][o],
// the shortcut's x_1x1 (x) dy, and (it == 0) db2 / db1 as ones (x) dz / dy; 4 pixels per MFMA step
__global__ __launch_bounds__(256) void k_trans_wgrad_mfma(const float* __restrict__ dy, const uint8_t* __restrict__ mask,
                                                          const float* __restrict__ x, float* __restrict__ part, int N,
                                                          int H, int W, int Ci, int Co, int S, int Ho, int Wo, int pt,
                                                          int pl, int px_per_chunk, int chunks) {
  const int IT = Ci / 16, OT = Co / 16;
  const long task = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (task >= (long)chunks * IT * OT) return;
  const int lane = threadIdx.x & 63, g = lane >> 4, lx = lane & 15;
  const int ot = (int)(task % OT), it = (int)((task / OT) % IT), chunk = (int)(task / ((long)OT * IT));
  const long P = (long)N * Ho * Wo;
  const long p0 = (long)chunk * px_per_chunk, p1 = min(P, p0 + px_per_chunk);
  f32x4 acc[kTK * kTK + 1], accb2 = {0.f, 0.f, 0.f, 0.f}, accb1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t <= kTK * kTK; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int ci = 16 * it + lx, co = 16 * ot + lx;  // A row (input channel), B column (output channel)
#pragma unroll 2
  for (long pb = p0; pb < p1; pb += 4) {
    const long p = pb + g;  // this lane group's pixel of the step
    const bool pin = p < p1;
    const long pc = pin ? p : p0;
    const int xo = (int)(pc % Wo), yo = (int)((pc / Wo) % Ho), n = (int)(pc / ((long)Wo * Ho));
    const float dyv = pin ? dy[pc * Co + co] : 0.f;
    const float dzv = (pin && mask[pc * Co + co]) ? dyv : 0.f;
#pragma unroll
    for (int ky = 0; ky < kTK; ++ky) {
      const int gy = S * yo + ky - pt;
#pragma unroll
      for (int kx = 0; kx < kTK; ++kx) {
        const int gx = S * xo + kx - pl;
        const bool ok = pin && gy >= 0 && gy < H && gx >= 0 && gx < W;
        const float xv = ok ? x[(((long)n * H + gy) * W + gx) * Ci + ci] : 0.f;
        acc[ky * kTK + kx] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv, dzv, acc[ky * kTK + kx], 0, 0, 0);
      }
    }
    const float xs = pin ? x[(((long)n * H + S * yo) * W + S * xo) * Ci + ci] : 0.f;
    acc[kTK * kTK] = __builtin_amdgcn_mfma_f32_16x16x4f32(xs, dyv, acc[kTK * kTK], 0, 0, 0);
    if (it == 0) {  // (wave-uniform)
      accb2 = __builtin_amdgcn_mfma_f32_16x16x4f32(1.f, dzv, accb2, 0, 0, 0);
      accb1 = __builtin_amdgcn_mfma_f32_16x16x4f32(1.f, dyv, accb1, 0, 0, 0);
    }
  }
  const long E2 = (long)kTK * kTK * Ci * Co, E1 = (long)Ci * Co, ET = E2 + Co + E1 + Co;
  float* out = part + (long)chunk * ET;
#pragma unroll
  for (int t = 0; t < kTK * kTK; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) out[((long)t * Ci + 16 * it + 4 * g + j) * Co + co] = acc[t][j];
#pragma unroll
  for (int j = 0; j < 4; ++j) out[E2 + Co + (long)(16 * it + 4 * g + j) * Co + co] = acc[kTK * kTK][j];
  if (it == 0 && g == 0) {  // every accumulator row of ones (x) dz is the column sum
    out[E2 + co] = accb2[0];
    out[E2 + Co + E1 + co] = accb1[0];
  }
}

// ---------------------------------------------------------------------------
// The stride-2 transition's weight gradient with LDS-staged operands
// (k_trans_wgrad_lds; even H and W, so TF's 'same' padding puts no row / column
// before the image: output (yo, xo) reads input rows 2yo .. 2yo+2, columns
// 2xo .. 2xo+2, and the 1x1 shortcut reads (2yo, 2xo) = tap 0's position).
// A workgroup (8 waves) stages a band of BRO = 4 output rows: the 2 BRO + 1
// input rows (W + 1 columns, zeros past the image) and the band's dy and
// dz = dy [z > 0], pixel strides padded (x: CI + 8 floats, so the lane groups'
// even pixels of a half fall on disjoint banks; dy / dz: CO + 16 when CO is a
// multiple of 32).  Waves = (i-tile, o-tile) pair x RS k-step splits; K = 4
// output pixels per v_mfma_f32_16x16x4_f32; a wave holds the 9 taps + the 1x1
// (sharing tap 0's A operand) and, at it = 0, db2 / db1 (ones x dz / dy).
// Persistent over bands; the RS partials summed through LDS, one partial slab
// [dK2 | db2 | dK1 | db1] per workgroup, summed by k_sum_chunks.
// ---------------------------------------------------------------------------
template <int CI, int CO, int WO>
struct TWg {
  static constexpr int IT = CI / 16, OT = CO / 16, P = IT * OT, NW = 8, RS = NW / P, BRO = 4, XR = 2 * BRO + 1;
  static constexpr int TW = 2 * WO + 1, XS = CI + 8, DS = CO % 32 == 0 ? CO + 16 : CO, NPX = BRO * WO;
  static constexpr int XF = XR * TW * XS, DF = NPX * DS, ACC = 12;
  static constexpr size_t LDS = std::max((size_t)(XF + 2 * DF) * 4, RS > 1 ? (size_t)P * ACC * 256 * 4 : (size_t)0);
  static_assert(P * RS == NW, "transition wgrad: IT x OT must divide 8");
};

template <int CI, int CO, int WO, typename T>
__global__ __launch_bounds__(512) void k_trans_wgrad_lds(const T* __restrict__ dy, const uint8_t* __restrict__ mask,
                                                         const T* __restrict__ x, float* __restrict__ part, int N,
                                                         int H) {
  using G = TWg<CI, CO, WO>;
  constexpr int W = 2 * WO, TW = G::TW, XS = G::XS, DS = G::DS, BRO = G::BRO;
  extern __shared__ __attribute__((aligned(16))) float lds_tw[];
  float* xt = lds_tw;              // [XR][TW][XS]
  float* dzt = lds_tw + G::XF;     // [NPX][DS]
  float* dyt = dzt + G::DF;        // [NPX][DS]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, lx = lane & 15;
  const int pr = wave % G::P, rs = wave / G::P, it = pr / G::OT, ot = pr % G::OT;
  const int Ho = H / 2, nb = (Ho + BRO - 1) / BRO;
  const long items = (long)N * nb;
  const long i0 = (long)blockIdx.x * items / gridDim.x, i1 = (long)(blockIdx.x + 1) * items / gridDim.x;
  f32x4 acc[10], accb2 = {0.f, 0.f, 0.f, 0.f}, accb1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 10; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (long item = i0; item < i1; ++item) {
    const int n = (int)(item / nb), yo0 = (int)(item % nb) * BRO;
    const int rows = min(BRO, Ho - yo0);
    __syncthreads();  // the previous band's operands consumed
    // (staged BS elements at a time, all loads before their stores: a rolled loop waited for each)
    stage_batched<G::XR * TW * (CI / 4), 512>(tid, [&](int i, f32x4& v, unsigned&) {
      const int j = i / (TW * (CI / 4)), rem = i % (TW * (CI / 4)), col = rem / (CI / 4), c4 = rem % (CI / 4);
      const int gy = 2 * yo0 + j;
      if (gy < H && col < W) v = ld4(x + (((long)n * H + gy) * W + col) * CI + 4 * c4);
    }, [&](int i, const f32x4& v, unsigned) {
      const int j = i / (TW * (CI / 4)), rem = i % (TW * (CI / 4)), col = rem / (CI / 4), c4 = rem % (CI / 4);
      *(f32x4*)(xt + (j * TW + col) * XS + 4 * c4) = v;
    });
    stage_batched<G::NPX * (CO / 4), 512>(tid, [&](int i, f32x4& v, unsigned& m) {
      const int k = i / (CO / 4), c4 = i % (CO / 4);
      if (k / WO < rows) {
        const long e = (((long)n * Ho + yo0) * WO + k) * CO + 4 * c4;
        v = ld4(dy + e);
        m = *(const unsigned*)(mask + e);
      }
    }, [&](int i, const f32x4& v, unsigned m) {
      const int k = i / (CO / 4), c4 = i % (CO / 4);
      *(f32x4*)(dyt + k * DS + 4 * c4) = v;
      *(f32x4*)(dzt + k * DS + 4 * c4) = v * mask4u(m);
    });
    __syncthreads();
    const int steps = rows * WO / 4;
    for (int st = rs; st < steps; st += G::RS) {
      const int k = 4 * st + g, r = k / WO, xo = k % WO;
      const float bz = dzt[k * DS + 16 * ot + lx], by = dyt[k * DS + 16 * ot + lx];
      const float* xa = xt + ((2 * r) * TW + 2 * xo) * XS + 16 * it + lx;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const float a = xa[((t / 3) * TW + t % 3) * XS];
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bz, acc[t], 0, 0, 0);
        if (t == 0) acc[9] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, by, acc[9], 0, 0, 0);
      }
      if (it == 0) {  // (wave-uniform)
        accb2 = __builtin_amdgcn_mfma_f32_16x16x4f32(1.f, bz, accb2, 0, 0, 0);
        accb1 = __builtin_amdgcn_mfma_f32_16x16x4f32(1.f, by, accb1, 0, 0, 0);
      }
    }
  }
  mfma_f32_settle();  // (the result is read below: every path sees the wait states)
  if constexpr (G::RS > 1) {  // the k-step splits' partials, one split at a time, fixed order
    float* mine = lds_tw + (long)pr * G::ACC * 256;
#pragma unroll 1
    for (int src = 1; src < G::RS; ++src) {
      __syncthreads();
      if (rs == src) {
#pragma unroll
        for (int t = 0; t < 10; ++t) *(f32x4*)(mine + (t * 64 + lane) * 4) = acc[t];
        *(f32x4*)(mine + (10 * 64 + lane) * 4) = accb2;
        *(f32x4*)(mine + (11 * 64 + lane) * 4) = accb1;
      }
      __syncthreads();
      if (rs == 0) {
#pragma unroll
        for (int t = 0; t < 10; ++t) acc[t] += *(const f32x4*)(mine + (t * 64 + lane) * 4);
        accb2 += *(const f32x4*)(mine + (10 * 64 + lane) * 4);
        accb1 += *(const f32x4*)(mine + (11 * 64 + lane) * 4);
      }
    }
  }
  if (rs != 0) return;
  constexpr long E2 = 9L * CI * CO, E1 = (long)CI * CO, ET = E2 + CO + E1 + CO;
  float* out = part + (long)blockIdx.x * ET;
  const int co = 16 * ot + lx;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) out[((long)t * CI + 16 * it + 4 * g + j) * CO + co] = acc[t][j];
#pragma unroll
  for (int j = 0; j < 4; ++j) out[E2 + CO + (long)(16 * it + 4 * g + j) * CO + co] = acc[9][j];
  if (it == 0 && g == 0) {
    out[E2 + co] = accb2[0];
    out[E2 + CO + E1 + co] = accb1[0];
  }
}

// The stride-2 transition's forward with LDS-staged input rows (k_trans_fwd_lds;
// H a multiple of 8, W in {32, 16}): a workgroup stages the 2 BRO + 1 input
// rows of a band of BRO = 4 output rows (W + 1 columns, the last zero; pixel
// stride CI + 4 floats), a wave = (o-tile, 16-pixel tile of the band) keeps its
// K2 / K1 fragments in registers: D[o][pixel] over (tap, i), the 1x1 shortcut
// from tap 0's operand, y = relu(z) + shortcut and the relu mask bytes in the
// epilogue.  T = bf16 for the bf16 nets (the activations in and out in bf16,
// staged and computed in fp32), float otherwise.
template <int CI, int CO, int WO>
struct TFw {
  static constexpr int W = 2 * WO, OT = CO / 16, IQ = CI / 16, BRO = 4, XR = 2 * BRO + 1, TW = W + 1, PX = CI + 4;
  static constexpr int PT = BRO * WO / 16, NW = OT * PT, XF = XR * TW * PX;
  static constexpr size_t LDS = (size_t)XF * 4;
};

template <int CI, int CO, int WO, typename T>
__global__ __launch_bounds__((64 * TFw<CI, CO, WO>::NW)) void k_trans_fwd_lds(
    const T* __restrict__ x, T* __restrict__ y, uint8_t* __restrict__ mask, const float* __restrict__ k2,
    const float* __restrict__ b2, const float* __restrict__ k1, const float* __restrict__ b1, int N, int H) {
  using G = TFw<CI, CO, WO>;
  constexpr int W = G::W, TW = G::TW, PX = G::PX, BRO = G::BRO, IQ = G::IQ;
  extern __shared__ __attribute__((aligned(16))) float lds_tf[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, lx = lane & 15;
  const int ot = wave % G::OT, pt = wave / G::OT;
  const int Ho = H / 2, nb = Ho / BRO;
  const long items = (long)N * nb;
  const long i0 = (long)blockIdx.x * items / gridDim.x, i1 = (long)(blockIdx.x + 1) * items / gridDim.x;
  // A = K^T fragments of o-tile ot: lane (lx, g), k-step s of i-group q: i = 16q + 4g + s, o = 16 ot + lx
  float A2[9][IQ][4], A1[IQ][4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int q = 0; q < IQ; ++q)
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) A2[t][q][s4] = k2[((long)t * CI + 16 * q + 4 * g + s4) * CO + 16 * ot + lx];
#pragma unroll
  for (int q = 0; q < IQ; ++q)
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) A1[q][s4] = k1[(long)(16 * q + 4 * g + s4) * CO + 16 * ot + lx];
  const int o0 = 16 * ot + 4 * g;  // the lane's 4 output channels (accumulator rows)
  const f32x4 bb2 = ld4(b2 + o0), bb1 = ld4(b1 + o0);
  const int p = 16 * pt + lx, r = p / WO, xo = p % WO;  // the lane's output pixel in the band
  for (long item = i0; item < i1; ++item) {
    const int n = (int)(item / nb), yo0 = (int)(item % nb) * BRO;
    __syncthreads();  // the previous band's rows consumed
    stage_batched<G::XR * TW * (CI / 4), 64 * G::NW>(tid, [&](int e, f32x4& v, unsigned&) {
      const int j = e / (TW * (CI / 4)), rem = e % (TW * (CI / 4)), col = rem / (CI / 4), c4 = rem % (CI / 4);
      const int gy = 2 * yo0 + j;
      if (gy < H && col < W) v = ld4(x + (((long)n * H + gy) * W + col) * CI + 4 * c4);
    }, [&](int e, const f32x4& v, unsigned) {
      const int j = e / (TW * (CI / 4)), rem = e % (TW * (CI / 4)), col = rem / (CI / 4), c4 = rem % (CI / 4);
      *(f32x4*)(lds_tf + (j * TW + col) * PX + 4 * c4) = v;
    });
    __syncthreads();
    f32x4 acc = {0.f, 0.f, 0.f, 0.f}, accs = {0.f, 0.f, 0.f, 0.f};
    const float* xb = lds_tf + ((2 * r) * TW + 2 * xo) * PX + 4 * g;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int q = 0; q < IQ; ++q) {
        const f32x4 bv = *(const f32x4*)(xb + ((t / 3) * TW + t % 3) * PX + 16 * q);
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A2[t][q][s4], bv[s4], acc, 0, 0, 0);
          if (t == 0) accs = __builtin_amdgcn_mfma_f32_16x16x4f32(A1[q][s4], bv[s4], accs, 0, 0, 0);
        }
      }
    mfma_f32_settle();
    const long pg = ((long)n * Ho + yo0 + r) * WO + xo;
    f32x4 v;
    unsigned mb = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float z = acc[j] + bb2[j];
      v[j] = fmaxf(z, 0.f) + (accs[j] + bb1[j]);
      mb |= (z > 0.f ? 1u : 0u) << (8 * j);
    }
    st4(y + pg * CO + o0, v);
    if (mask) *(unsigned*)(mask + pg * CO + o0) = mb;
  }
}

// the LDS-staged transition kernels' shapes (forward, input and weight gradients)
bool trans_lds_supported(int H, int W, int Ci, int Co, int S) {
  if (S != 2 || H % 8 || (W != 32 && W != 16)) return false;
  return (Ci == 16 && (Co == 16 || Co == 32)) || (Ci == 32 && (Co == 32 || Co == 64));
}

template <int CI, int CO, int WO, typename T>
int launch_trans_fwd_lds(const T* x, T* y, uint8_t* mask, const float* k2, const float* b2, const float* k1,
                         const float* b1, int N, int H, hipStream_t s) {
  using G = TFw<CI, CO, WO>;
  const long items = (long)N * (H / 2 / G::BRO);
  int cus = cu_count();
  if (cus <= 0) cus = 256;
  const int grid = (int)std::max<long>(1, std::min<long>(items, 2L * cus));  // 2 workgroups per CU
  hipLaunchKernelGGL((k_trans_fwd_lds<CI, CO, WO, T>), dim3(grid), dim3(64 * G::NW), G::LDS, s, x, y, mask, k2, b2, k1,
                     b1, N, H);
  ASR_LAUNCH_CHECK("k_trans_fwd_lds");
  return ASR_OK;
}

int trans_fwd_lds(const void* x, void* y, uint8_t* mask, const float* k2, const float* b2, const float* k1,
                  const float* b1, int act_bf16, int N, int H, int W, int Ci, int Co, hipStream_t s) {
#define ASR_TFL(CI_, CO_, WO_)                                                                                       \
  if (Ci == CI_ && Co == CO_ && W == 2 * WO_)                                                                        \
    return act_bf16 ? launch_trans_fwd_lds<CI_, CO_, WO_>((const bf16*)x, (bf16*)y, mask, k2, b2, k1, b1, N, H, s)   \
                    : launch_trans_fwd_lds<CI_, CO_, WO_>((const float*)x, (float*)y, mask, k2, b2, k1, b1, N, H, s);
  ASR_TFL(16, 16, 16) ASR_TFL(16, 32, 16) ASR_TFL(32, 32, 16) ASR_TFL(32, 64, 16)
  ASR_TFL(16, 16, 8) ASR_TFL(16, 32, 8) ASR_TFL(32, 32, 8) ASR_TFL(32, 64, 8)
#undef ASR_TFL
  return fail(ASR_E_UNSUPPORTED, "transition forward (LDS): Ci=%d Co=%d W=%d", Ci, Co, W);
}

// The stride-2 transition's input gradient with LDS-staged operands
// (k_trans_dgrad_lds; even H and W).  dx[gy][gx] = sum over the taps with
// gy - ky, gx - kx even of K2[ky][kx] dz[(gy-ky)/2][(gx-kx)/2] (+ K1 dy[gy/2][gx/2]
// at even gy, gx): by the parities of (gy, gx) the output splits into four
// classes with 4 (+ the 1x1), 2, 2 and 1 taps, and a 16-pixel MFMA tile holds
// pixels of one class (one row's 16 even or odd columns at W = 32; two rows
// gy, gy + 2 of 8 such columns at W = 16), so no MFMA multiplies a structural
// zero.  A workgroup (8 waves) stages a band of BR = 8 output rows' operands:
// dz = dy [z > 0] and dy on the BR / 2 + 1 source rows x WO + 1 columns
// (source row / column -1 as zeros), pixel stride CO + 4 floats (the 16
// lanes' 16-B reads on disjoint banks).  A wave keeps its i-tile's K2 / K1
// fragments in registers and takes the band's (row group, column parity)
// tiles round-robin; v_mfma_f32_16x16x4_f32, D = dx tile [i][pixel].
template <int CI, int CO, int WO>
struct TDg {
  static constexpr int W = 2 * WO, IT = CI / 16, OQ = CO / 16, BR = 8, SR = BR / 2 + 1, SC = WO + 1;
  static constexpr int PS = CO + 4, SF = SR * SC * PS;       // floats per staged tile
  static constexpr int RPT = W == 32 ? 1 : 2;                // rows per MFMA tile (W/2 columns each)
  static constexpr int TPB = (BR / RPT) * 2;                 // (row group, column parity) tiles per band per i-tile
  static constexpr int NW = 8, WPI = NW / IT;                // waves per i-tile
  static constexpr size_t LDS = (size_t)2 * SF * 4;
  static_assert(W == 32 || W == 16, "transition dgrad (LDS): W in {32, 16}");
  static_assert(NW % IT == 0, "transition dgrad (LDS): CI / 16 must divide 8");
};

template <int CI, int CO, int WO, typename T>
__global__ __launch_bounds__(512) void k_trans_dgrad_lds(const T* __restrict__ dy, const uint8_t* __restrict__ mask,
                                                         const float* __restrict__ k2, const float* __restrict__ k1,
                                                         T* __restrict__ dx, int N, int H) {
  using G = TDg<CI, CO, WO>;
  constexpr int W = G::W, BR = G::BR, SC = G::SC, PS = G::PS, OQ = G::OQ;
  extern __shared__ __attribute__((aligned(16))) float lds_td[];
  float* dzt = lds_td;          // [SR][SC][PS]
  float* dyt = lds_td + G::SF;  // [SR][SC][PS]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, lx = lane & 15;
  const int it = wave / G::WPI, wi = wave % G::WPI;
  const int Ho = H / 2, nb = H / BR;
  const long items = (long)N * nb;
  const long i0 = (long)blockIdx.x * items / gridDim.x, i1 = (long)(blockIdx.x + 1) * items / gridDim.x;
  // A = K2[tap][i][o]^T fragments of i-tile it: lane (lx, g), k-step s of o-group q: o = 16q + 4g + s
  float A2[9][OQ][4], A1[OQ][4];
  const int i = 16 * it + lx;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int q = 0; q < OQ; ++q) {
      const f32x4 v = ld4(k2 + ((long)t * CI + i) * CO + 16 * q + 4 * g);
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) A2[t][q][s4] = v[s4];
    }
#pragma unroll
  for (int q = 0; q < OQ; ++q) {
    const f32x4 v = ld4(k1 + (long)i * CO + 16 * q + 4 * g);
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) A1[q][s4] = v[s4];
  }
  for (long item = i0; item < i1; ++item) {
    const int n = (int)(item / nb), gy0 = (int)(item % nb) * BR, yb = gy0 / 2 - 1;  // staged source row 0 = yo yb
    __syncthreads();  // the previous band's operands consumed
    stage_batched<G::SR * SC * (CO / 4), 512>(tid, [&](int e, f32x4& v, unsigned& m) {
      const int j = e / (SC * (CO / 4)), rem = e % (SC * (CO / 4)), c = rem / (CO / 4), c4 = rem % (CO / 4);
      const int yo = yb + j, xo = c - 1;
      if (yo >= 0 && yo < Ho && xo >= 0) {
        const long off = (((long)n * Ho + yo) * WO + xo) * CO + 4 * c4;
        v = ld4(dy + off);
        m = *(const unsigned*)(mask + off);
      }
    }, [&](int e, const f32x4& v, unsigned m) {
      const int j = e / (SC * (CO / 4)), rem = e % (SC * (CO / 4)), c = rem / (CO / 4), c4 = rem % (CO / 4);
      *(f32x4*)(dyt + (j * SC + c) * PS + 4 * c4) = v;
      *(f32x4*)(dzt + (j * SC + c) * PS + 4 * c4) = v * mask4u(m);
    });
    __syncthreads();
    for (int tk = wi; tk < G::TPB; tk += G::WPI) {  // (wave-uniform)
      const int pxp = tk & 1, rg = tk >> 1;          // column parity, row group
      // row group rg: W = 32 one row gy0 + rg; W = 16 rows {a, a + 2}, a = gy0 + (rg & 1) + 4 (rg >> 1)
      const int gyA = G::RPT == 1 ? gy0 + rg : gy0 + (rg & 1) + 4 * (rg >> 1);
      const int gy = gyA + (G::RPT == 2 ? 2 * (lx / (W / 2)) : 0), gx = 2 * (lx % (W / 2)) + pxp;
      const int py = gyA & 1;  // (the same for both rows of a W = 16 tile)
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        if ((ky & 1) != py) continue;  // (wave-uniform)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          if ((kx & 1) != pxp) continue;  // (wave-uniform)
          const int j = (gy - ky) / 2 - yb, c = (gx - kx) / 2 + 1;  // ((gy - ky) even: exact halves, -1 allowed)
          const float* bp = dzt + (j * SC + c) * PS + 4 * g;
#pragma unroll
          for (int q = 0; q < OQ; ++q) {
            const f32x4 bv = *(const f32x4*)(bp + 16 * q);
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4)
              acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A2[3 * ky + kx][q][s4], bv[s4], acc, 0, 0, 0);
          }
        }
      }
      if (py == 0 && pxp == 0) {  // the 1x1 shortcut at even (gy, gx)
        const float* bp = dyt + ((gy / 2 - yb) * SC + gx / 2 + 1) * PS + 4 * g;
#pragma unroll
        for (int q = 0; q < OQ; ++q) {
          const f32x4 bv = *(const f32x4*)(bp + 16 * q);
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A1[q][s4], bv[s4], acc, 0, 0, 0);
        }
      }
      mfma_f32_settle();
      st4(dx + (((long)n * H + gy) * W + gx) * CI + 16 * it + 4 * g, acc);
    }
  }
}


template <int CI, int CO, int WO, typename T>
int launch_trans_dgrad_lds(const T* dy, const uint8_t* mask, const float* k2, const float* k1, T* dx, int N,
                           int H, hipStream_t s) {
  using G = TDg<CI, CO, WO>;
  const long items = (long)N * (H / G::BR);
  int cus = cu_count();
  if (cus <= 0) cus = 256;
  const int grid = (int)std::max<long>(1, std::min<long>(items, (long)cus));  // 1 workgroup per CU
  hipLaunchKernelGGL((k_trans_dgrad_lds<CI, CO, WO, T>), dim3(grid), dim3(512), G::LDS, s, dy, mask, k2, k1, dx, N, H);
  ASR_LAUNCH_CHECK("k_trans_dgrad_lds");
  return ASR_OK;
}

int trans_dgrad_lds(const void* dy, const uint8_t* mask, const float* k2, const float* k1, void* dx, int act_bf16, int N,
                    int H, int W, int Ci, int Co, hipStream_t s) {
#define ASR_TDL(CI_, CO_, WO_)                                                                                       \
  if (Ci == CI_ && Co == CO_ && W == 2 * WO_)                                                                        \
    return act_bf16 ? launch_trans_dgrad_lds<CI_, CO_, WO_>((const bf16*)dy, mask, k2, k1, (bf16*)dx, N, H, s)       \
                    : launch_trans_dgrad_lds<CI_, CO_, WO_>((const float*)dy, mask, k2, k1, (float*)dx, N, H, s);
  ASR_TDL(16, 16, 16) ASR_TDL(16, 32, 16) ASR_TDL(32, 32, 16) ASR_TDL(32, 64, 16)
  ASR_TDL(16, 16, 8) ASR_TDL(16, 32, 8) ASR_TDL(32, 32, 8) ASR_TDL(32, 64, 8)
#undef ASR_TDL
  return fail(ASR_E_UNSUPPORTED, "transition dgrad (LDS): Ci=%d Co=%d W=%d", Ci, Co, W);
}

// the LDS-staged weight gradient's shapes: stride 2, even H / W, W/2 in {16, 8}, (Ci, Co) pairs with IT x OT <= 8
bool trans_wgrad_lds_supported(int H, int W, int Ci, int Co, int S) {
  if (S != 2 || (H & 1) || (W & 1) || (W != 32 && W != 16)) return false;
  return (Ci == 16 && (Co == 16 || Co == 32)) || (Ci == 32 && (Co == 32 || Co == 64));
}

template <int CI, int CO, int WO, typename T>
int launch_trans_wgrad_lds(const T* dy, const uint8_t* mask, const T* x, float* part, int N, int H,
                           int max_rows, int* rows_out, hipStream_t s) {
  using G = TWg<CI, CO, WO>;
  const long items = (long)N * ((H / 2 + G::BRO - 1) / G::BRO);
  int cus = cu_count();
  if (cus <= 0) cus = 256;
  const int grid = (int)std::max<long>(1, std::min<long>({items, 2L * cus, (long)max_rows}));  // 2 per CU
  hipLaunchKernelGGL((k_trans_wgrad_lds<CI, CO, WO, T>), dim3(grid), dim3(512), G::LDS, s, dy, mask, x, part, N, H);
  ASR_LAUNCH_CHECK("k_trans_wgrad_lds");
  *rows_out = grid;
  return ASR_OK;
}

// act_bf16: dy and x are the bf16 net's activations (bf16), else fp32
int trans_wgrad_lds(const void* dy, const uint8_t* mask, const void* x, int act_bf16, float* part, int N, int H, int W,
                    int Ci, int Co, int max_rows, int* rows, hipStream_t s) {
#define ASR_TWL(CI_, CO_, WO_)                                                                                        \
  if (Ci == CI_ && Co == CO_ && W == 2 * WO_)                                                                         \
    return act_bf16 ? launch_trans_wgrad_lds<CI_, CO_, WO_>((const bf16*)dy, mask, (const bf16*)x, part, N, H,        \
                                                            max_rows, rows, s)                                        \
                    : launch_trans_wgrad_lds<CI_, CO_, WO_>((const float*)dy, mask, (const float*)x, part, N, H,      \
                                                            max_rows, rows, s);
  ASR_TWL(16, 16, 16) ASR_TWL(16, 32, 16) ASR_TWL(32, 32, 16) ASR_TWL(32, 64, 16)
  ASR_TWL(16, 16, 8) ASR_TWL(16, 32, 8) ASR_TWL(32, 32, 8) ASR_TWL(32, 64, 8)
#undef ASR_TWL
  return fail(ASR_E_UNSUPPORTED, "transition wgrad (LDS): Ci=%d Co=%d W=%d", Ci, Co, W);
}

bool trans_mfma(int Ci, int Co) { return Ci % 16 == 0 && Co % 16 == 0; }

// MFMA weight gradient: chunks of ppc output pixels (a multiple of 4) such that about 2048 waves
// run, each over few pixel steps (the steps are gather-latency bound)
int trans_mfma_chunks(int N, int Ho, int Wo, int Ci, int Co, int* ppc) {
  const long P = (long)N * Ho * Wo;
  const long target = std::max(1, 2048 / ((Ci / 16) * (Co / 16)));
  *ppc = (int)std::max<long>(16, ((P + target - 1) / target + 3) / 4 * 4);
  return (int)((P + *ppc - 1) / *ppc);
}

int trans_chunks(int N, int Ho, int* rpc) {
  const long R = (long)N * Ho;
  const long chunks = std::max<long>(1, std::min<long>(R, kMaxTransChunks));
  *rpc = (int)((R + chunks - 1) / chunks);
  return (int)((R + *rpc - 1) / *rpc);
}

int check_trans(int N, int H, int W, int Ci, int Co, int S) {
  if (N < 1 || H < 1 || W < 1 || Ci < 1 || Co < 1 || (S != 1 && S != 2))
    return fail(ASR_E_ARG, "transition: bad shape N=%d H=%d W=%d Ci=%d Co=%d stride=%d", N, H, W, Ci, Co, S);
  if ((long)N * H * W * std::max(Ci, Co) > (1L << 40)) return fail(ASR_E_ARG, "transition: shape too large");
  return ASR_OK;
}

int trans_forward(const float* x, float* y, uint8_t* mask, const float* k2, const float* b2, const float* k1,
                  const float* b1, int N, int H, int W, int Ci, int Co, int S, hipStream_t s) {
  const TGeom g = tgeom(H, W, S);
  const long tasks = (long)N * g.Ho * ((g.Wo + 15) / 16) * ((Co + 15) / 16);
  const long blocks = (tasks + 3) / 4;
  if (blocks > 0x7fffffffL) return fail(ASR_E_ARG, "transition: problem too large");
  if (trans_lds_supported(H, W, Ci, Co, S)) return trans_fwd_lds(x, y, mask, k2, b2, k1, b1, 0, N, H, W, Ci, Co, s);
  if (trans_mfma(Ci, Co)) {
    hipLaunchKernelGGL(k_trans_fwd_mfma, dim3((unsigned)blocks), dim3(256), 0, s, x, y, mask, k2, b2, k1, b1, N, H,
                       W, Ci, Co, S, g.Ho, g.Wo, g.pt, g.pl);
    ASR_LAUNCH_CHECK("k_trans_fwd_mfma");
    return ASR_OK;
  }
  hipLaunchKernelGGL(k_trans_fwd, dim3((unsigned)blocks), dim3(256), 0, s, x, y, mask, k2, b2, k1, b1, N, H, W, Ci,
                     Co, S, g.Ho, g.Wo, g.pt, g.pl);
  ASR_LAUNCH_CHECK("k_trans_fwd");
  return ASR_OK;
}

size_t trans_ws_bytes(int N, int H, int W, int Ci, int Co, int S) {
  const TGeom g = tgeom(H, W, S);
  int rpc = 0;
  const int nch = trans_mfma(Ci, Co) ? trans_mfma_chunks(N, g.Ho, g.Wo, Ci, Co, &rpc) : trans_chunks(N, g.Ho, &rpc);
  return align_up((size_t)nch * trans_param_floats(Ci, Co) * 4, 256);
}

// the bf16 nets' transition backward on the LDS kernels (trans_lds_supported shapes): dy, x and dx in bf16
int trans_backward_bf16(const bf16* dy, const bf16* x, const uint8_t* mask, const float* k2, const float* k1, int N,
                        int H, int W, int Ci, int Co, int S, bf16* dx, float* dparams, float* part, hipStream_t s) {
  if (!trans_lds_supported(H, W, Ci, Co, S)) return fail(ASR_E_UNSUPPORTED, "transition (bf16): shape");
  const TGeom g = tgeom(H, W, S);
  ASR_TRY(trans_dgrad_lds(dy, mask, k2, k1, dx, 1, N, H, W, Ci, Co, s));
  int ppc = 0;
  int rows = trans_mfma_chunks(N, g.Ho, g.Wo, Ci, Co, &ppc);  // (the workspace's partial rows, trans_ws_bytes)
  ASR_TRY(trans_wgrad_lds(dy, mask, x, 1, part, N, H, W, Ci, Co, rows, &rows, s));
  const long ET = trans_param_floats(Ci, Co);
  hipLaunchKernelGGL(k_sum_chunks, dim3((unsigned)((ET + 63) / 64)), dim3(256), 0, s, part, rows, ET, dparams);
  ASR_LAUNCH_CHECK("k_sum_chunks");
  return ASR_OK;
}

int trans_backward(const float* dy, const float* x, const uint8_t* mask, const float* k2, const float* k1, int N,
                   int H, int W, int Ci, int Co, int S, float* dx, float* dparams, float* part, hipStream_t s) {
  const TGeom g = tgeom(H, W, S);
  if (trans_mfma(Ci, Co)) {
    if (dx && trans_lds_supported(H, W, Ci, Co, S)) {
      ASR_TRY(trans_dgrad_lds(dy, mask, k2, k1, dx, 0, N, H, W, Ci, Co, s));
    } else if (dx) {
      const long blocks = ((long)N * H * ((W + 15) / 16) * (Ci / 16) + 3) / 4;
      if (blocks > 0x7fffffffL) return fail(ASR_E_ARG, "transition: problem too large");
      hipLaunchKernelGGL(k_trans_dgrad_mfma, dim3((unsigned)blocks), dim3(256), 0, s, dy, mask, k2, k1, dx, N, H, W,
                         Ci, Co, S, g.Ho, g.Wo, g.pt, g.pl);
      ASR_LAUNCH_CHECK("k_trans_dgrad_mfma");
    }
    if (dparams) {
      int ppc = 0;
      int chunks = trans_mfma_chunks(N, g.Ho, g.Wo, Ci, Co, &ppc);  // (the workspace's partial rows)
      const long ET = trans_param_floats(Ci, Co);
      if (trans_wgrad_lds_supported(H, W, Ci, Co, S)) {
        ASR_TRY(trans_wgrad_lds(dy, mask, x, 0, part, N, H, W, Ci, Co, chunks, &chunks, s));
      } else {
        const long blocks = ((long)chunks * (Ci / 16) * (Co / 16) + 3) / 4;
        hipLaunchKernelGGL(k_trans_wgrad_mfma, dim3((unsigned)blocks), dim3(256), 0, s, dy, mask, x, part, N, H, W,
                           Ci, Co, S, g.Ho, g.Wo, g.pt, g.pl, ppc, chunks);
        ASR_LAUNCH_CHECK("k_trans_wgrad_mfma");
      }
      hipLaunchKernelGGL(k_sum_chunks, dim3((unsigned)((ET + 63) / 64)), dim3(256), 0, s, part, chunks, ET, dparams);
      ASR_LAUNCH_CHECK("k_sum_chunks");
    }
    return ASR_OK;
  }
  if (dx) {
    const long total = (long)N * H * W * Ci;
    const unsigned grid = (unsigned)std::max<long>(1, std::min<long>((total + 255) / 256, 65536));
    hipLaunchKernelGGL(k_trans_dgrad, dim3(grid), dim3(256), 0, s, dy, mask, k2, k1, dx, N, H, W, Ci, Co, S, g.Ho,
                       g.Wo, g.pt, g.pl);
    ASR_LAUNCH_CHECK("k_trans_dgrad");
  }
  if (dparams) {
    int rpc = 0;
    const int nch = trans_chunks(N, g.Ho, &rpc);
    const long ET = trans_param_floats(Ci, Co);
    hipLaunchKernelGGL(k_trans_wgrad, dim3((unsigned)((ET + 255) / 256), nch), dim3(256), 0, s, dy, mask, x, part, N,
                       H, W, Ci, Co, S, g.Ho, g.Wo, g.pt, g.pl, rpc);
    ASR_LAUNCH_CHECK("k_trans_wgrad");
    hipLaunchKernelGGL(k_sum_chunks, dim3((unsigned)((ET + 63) / 64)), dim3(256), 0, s, part, nch, ET, dparams);
    ASR_LAUNCH_CHECK("k_sum_chunks");
  }
  return ASR_OK;
}

// ---------------------------------------------------------------------------
// the multi-stage executor
// ---------------------------------------------------------------------------
struct StageL {
  int C, L, H, W, S, Cp, Hp, Wp;  // S = 0: no transition; Cp/Hp/Wp the stage input's shape
  long P, ntheta, E, blk_stride, mask_bytes;
  long off_t, off_blk;          // parameter offsets (floats)
  size_t w_src, w_src_bwd, theta_dst, wbuf, wbuf_bwd, act_t, mask_t, acts, masks, grp, slabs;  // workspace offsets
  size_t act_tb, xin32;  // bf16 nets: the transition's output in bf16, its input in fp32 (kept for the backward)
  bool tdirect;          // bf16 nets: the transition on the LDS kernels in bf16 (no fp32 copies)
  bool deep;             // bf16 nets: a C = 16, 32 x 32 stage on the fused deep16 kernels (x0: its input slot,
  size_t x0;             //   followed by the L outputs at stride P, as deep16 reads them)
  bool img;              // bf16 nets: a 16 x 16 x 32 / 8 x 8 x 64 stage on the image-resident kernels
  bool img32;            // fp32 nets: the same on the fp32 image-resident kernels
  size_t dys;            //   its backward's per-layer input gradients (layers 0 .. L-2)
  long wstride;          // elements of one layer's W in wbuf (E fp32, or the bf16 MFMA pack)
  long grp_stride;   // floats per block of pass-1 group rows
  long slab_stride;  // floats per block of weight-gradient slabs
  int slab_rows;     // slab rows of one block's weight gradient (f32_block_slab_rows)
};
struct SLayout {
  int ns;
  StageL st[ASR_STAGES_MAX];
  bool sep_bwd;
  bool bf;              // bf16 activations / block convs (asr_stages_config.dtype)
  bool any_tconv;       // bf16 nets: a transition off the LDS kernels (fp32 copies and converts)
  int act_bytes;
  size_t t32a, t32b;    // bf16 nets: fp32 scratch of the transition backward (dy, dx)
  long off_c1k, off_c1b, off_fck, off_fcb, n_params, Pmax;
  size_t act0, probs, loss_per, dlogits, gap, dA, dB, cws, tws, sslabs, sred, total;
  size_t cws_bytes, tws_bytes, sred_bytes;
};

int stages_check(const asr_stages_config* c) {
  if (!c) return fail(ASR_E_ARG, "asr_stages: null config");
  if (c->N < 1 || c->H < 1 || c->W < 1 || c->num_classes < 1 || c->n_stages < 1 || c->n_stages > ASR_STAGES_MAX)
    return fail(ASR_E_ARG, "asr_stages: bad config (N=%d H=%d W=%d K=%d stages=%d)", c->N, c->H, c->W,
                c->num_classes, c->n_stages);
  if (c->param_kind < ASR_PARAM_3BY3 || c->param_kind > ASR_PARAM_REGULAR) return fail(ASR_E_ARG, "asr_stages: param_kind");
  if (c->stride[0] != 0) return fail(ASR_E_ARG, "asr_stages: stage 0 has no transition (stride[0] must be 0)");
  for (int s = 0; s < c->n_stages; ++s) {
    if (c->C[s] < 1 || c->L[s] < 0) return fail(ASR_E_ARG, "asr_stages: stage %d: C=%d L=%d", s, c->C[s], c->L[s]);
    if (s > 0 && c->stride[s] == 0 && c->C[s] != c->C[s - 1])
      return fail(ASR_E_ARG, "asr_stages: stage %d changes filters without a transition", s);
    if (s > 0 && c->stride[s] != 0 && c->stride[s] != 1 && c->stride[s] != 2)
      return fail(ASR_E_UNSUPPORTED, "asr_stages: stage %d: transition stride %d (1 or 2)", s, c->stride[s]);
  }
  if (!stem_supported(c->Cin, c->H, c->W, c->C[0]))
    return fail(ASR_E_UNSUPPORTED, "asr_stages: stem Cin=%d C=%d at %dx%d", c->Cin, c->C[0], c->H, c->W);
  if (c->C[c->n_stages - 1] > 256 || c->num_classes > 256)
    return fail(ASR_E_UNSUPPORTED, "asr_stages: head needs C and num_classes <= 256");
  if (c->use_norm && c->divide_by_stddev == 0.f) return fail(ASR_E_ARG, "asr_stages: divide_by_stddev == 0");
  if (c->dtype != ASR_F32 && c->dtype != ASR_BF16) return fail(ASR_E_ARG, "asr_stages: dtype %d", c->dtype);
  if (c->dtype == ASR_BF16) {
    int H = c->H, W = c->W;
    for (int s = 0; s < c->n_stages; ++s) {
      if (s > 0 && c->stride[s]) H = (H + c->stride[s] - 1) / c->stride[s], W = (W + c->stride[s] - 1) / c->stride[s];
      if (c->L[s] > 0 && !convb_supported(W, c->C[s]))
        return fail(ASR_E_UNSUPPORTED, "asr_stages: bf16 stage %d needs C in {16, 32, 64} and W in {32, 16, 8} (C=%d W=%d)",
                    s, c->C[s], W);
      if (c->C[s] % 8) return fail(ASR_E_UNSUPPORTED, "asr_stages: bf16 stage %d: C=%d not a multiple of 8", s, c->C[s]);
    }
  }
  return ASR_OK;
}

SLayout stages_layout(const asr_stages_config* c) {
  SLayout L{};
  L.ns = c->n_stages;
  L.sep_bwd = param_is_antisymmetric(c->param_kind, c->antisymmetric) == 0;
  L.bf = c->dtype == ASR_BF16;
  L.act_bytes = L.bf ? 2 : 4;
  // offset 0 is a reserved null page: a buffer offset left unassigned (0) can never alias a live
  // buffer, and stages_layout_valid rejects it
  size_t off = 256;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off += align_up(bytes, 256);
    return o;
  };
  long po = 0;
  L.off_c1k = po;
  po += 9L * c->Cin * c->C[0];
  L.off_c1b = po;
  po += c->C[0];
  int H = c->H, W = c->W, Cp = c->C[0];
  L.Pmax = (long)c->N * H * W * Cp;
  for (int s = 0; s < L.ns; ++s) {
    StageL& g = L.st[s];
    g.C = c->C[s];
    g.L = c->L[s];
    g.S = s > 0 ? c->stride[s] : 0;
    g.Cp = Cp;
    g.Hp = H;
    g.Wp = W;
    if (g.S) {
      const TGeom tg = tgeom(H, W, g.S);
      H = tg.Ho;
      W = tg.Wo;
    }
    g.H = H;
    g.W = W;
    g.P = (long)c->N * H * W * g.C;
    L.Pmax = std::max(L.Pmax, g.P);
    g.ntheta = theta_count(g.C, c->param_kind, c->antisymmetric);
    g.deep = c->dtype == ASR_BF16 && g.L > 0 && deep16_supported(H, W, g.C);
    g.img = c->dtype == ASR_BF16 && g.L > 0 && !g.deep && stage_img_supported(H, W, g.C);
    g.img32 = c->dtype != ASR_BF16 && g.L > 0 && stage_img32_supported(H, W, g.C);
    g.E = 9L * g.C * g.C;
    g.blk_stride = g.ntheta + g.C;
    g.mask_bytes = (long)align_up((size_t)asr_mask_bytes(c->N, H, W, g.C), 256);
    g.off_t = po;
    if (g.S) po += trans_param_floats(Cp, g.C);
    g.off_blk = po;
    po += (long)g.L * g.blk_stride;
    Cp = g.C;
  }
  L.off_fck = po;
  po += (long)Cp * c->num_classes;
  L.off_fcb = po;
  po += c->num_classes;
  L.n_params = po;
  // workspace
  if (!L.st[0].deep && !L.st[0].img && !L.st[0].img32)
    L.act0 = take((size_t)c->N * c->H * c->W * c->C[0] * L.act_bytes);
  L.cws_bytes = 0;
  L.tws_bytes = 0;
  for (int s = 0; s < L.ns; ++s) {
    StageL& g = L.st[s];
    g.w_src = take((size_t)g.E * 4);
    g.theta_dst = take((size_t)g.ntheta * 2 * 4);
    g.w_src_bwd = L.sep_bwd ? take((size_t)g.E * 4) : 0;
    g.wstride = L.bf ? asr_wpack_elems(g.C) : g.E;
    g.wbuf = take((size_t)std::max(g.L, 1) * g.wstride * L.act_bytes);
    g.wbuf_bwd = L.sep_bwd ? take((size_t)std::max(g.L, 1) * g.wstride * L.act_bytes) : 0;
    g.tdirect = L.bf && g.S && trans_lds_supported(g.Hp, g.Wp, g.Cp, g.C, g.S);
    L.any_tconv = L.any_tconv || (L.bf && g.S && !g.tdirect);
    if (g.deep || g.img || g.img32) {  // [x0 | x1 .. xL] contiguous; the stem or the transition writes x0 in place
      g.x0 = take((size_t)(g.L + 1) * g.P * L.act_bytes);
      g.acts = g.x0 + (size_t)g.P * L.act_bytes;
      if (s == 0) L.act0 = g.x0;
    }
    g.act_t = g.S && !g.tdirect ? (g.img32 ? g.x0 : take((size_t)g.P * 4)) : 0;  // (after x0: it may be x0)
    g.act_tb = g.S && L.bf ? ((g.deep || g.img) && g.tdirect ? g.x0 : take((size_t)g.P * 2)) : 0;
    g.xin32 = g.S && L.bf && !g.tdirect ? take((size_t)c->N * g.Hp * g.Wp * g.Cp * 4) : 0;
    g.mask_t = g.S ? take((size_t)g.P) : 0;
    if (!g.deep && !g.img && !g.img32) g.acts = take((size_t)std::max(g.L, 1) * g.P * L.act_bytes);
    g.masks = take((size_t)std::max(g.L, 1) * g.mask_bytes);
    g.dys = g.img || g.img32 ? take((size_t)g.L * g.P * L.act_bytes) : 0;
    // every block keeps its slabs until the stage's one reduction launch: sized by the
    // grid the fp32 weight gradient runs at this shape, not by the 512-row maximum
    // (deep16: its own slab rows per layer)
    g.slab_rows = g.deep ? (int)(deep16_slab_bytes(c->N, 1) / ((size_t)(g.E + g.C) * 4))
                         : f32_block_slab_rows(c->N, g.H, g.W, g.C);
    g.grp_stride = (long)reduce_groups(g.slab_rows) * (g.E + g.C);
    g.grp = take((size_t)std::max(g.L, 1) * g.grp_stride * 4);
    g.slab_stride = (long)g.slab_rows * (g.E + g.C);
    g.slabs = take(g.deep ? deep16_slab_bytes(c->N, g.L) : (size_t)g.L * g.slab_stride * 4);
    if (g.L > 0) L.cws_bytes = std::max(L.cws_bytes, asr_conv_backward_workspace_bytes(c->N, g.H, g.W, g.C, ASR_F32));
    if (g.S) L.tws_bytes = std::max(L.tws_bytes, trans_ws_bytes(c->N, g.Hp, g.Wp, g.Cp, g.C, g.S));
  }
  const int K = c->num_classes;
  L.probs = take((size_t)c->N * K * 4);
  L.loss_per = take((size_t)c->N * 4);
  L.dlogits = take((size_t)c->N * K * 4);
  L.gap = take((size_t)c->N * Cp * 4);
  L.dA = take((size_t)L.Pmax * 4);
  L.dB = take((size_t)L.Pmax * 4);
  L.cws = take(std::max<size_t>(L.cws_bytes, 256));
  L.tws = take(std::max<size_t>(L.tws_bytes, 256));
  L.t32a = L.any_tconv ? take((size_t)L.Pmax * 4) : 0;
  L.t32b = L.any_tconv ? take((size_t)L.Pmax * 4) : 0;
  const long E1 = 9L * c->Cin * c->C[0];
  L.sslabs = take((size_t)kMaxStemSlabs * (E1 + c->C[0]) * 4);
  L.sred_bytes = reduce_ws_bytes(kMaxStemSlabs, E1 + c->C[0]);
  L.sred = take(L.sred_bytes);
  L.total = off;
  return L;
}

// every buffer the executor will touch has an assigned (non-null) offset
bool stages_layout_valid(const SLayout& L) {
  if (!L.act0 || !L.probs || !L.dA || !L.dB || !L.sslabs) return false;
  for (int s = 0; s < L.ns; ++s) {
    const StageL& g = L.st[s];
    if (g.S && !g.mask_t) return false;
    if (g.S && !(L.bf ? g.act_tb : g.act_t)) return false;
    if (g.S && L.bf && !g.tdirect && (!g.act_t || !g.xin32)) return false;
    if (g.L > 0 && (!g.acts || !g.masks || !g.wbuf || !g.slabs || !g.grp)) return false;
    if ((g.deep || g.img || g.img32) && !g.x0) return false;
    if ((g.img || g.img32) && !g.dys) return false;
  }
  return true;
}

// forward through the stem and all stages; *xL = the last activation (fp32, or bf16 for a bf16 net)
int stages_forward_impl(const asr_stages_config* c, const SLayout& L, const float* params, const void* images,
                        bool training, unsigned char* b, hipStream_t s, const void** xL) {
  const float inv_std = c->use_norm ? 1.f / c->divide_by_stddev : 1.f;
  const int wdt = L.bf ? ASR_BF16 : ASR_F32;
  // every stage's W first, in one launch for the bf16 stages (the balanced pack of asr_theta_to_w,
  // k_theta_to_w_pack_bal: a workgroup per layer, the stages' packs side by side)
  PackJob jobs[kMaxPackJobs];
  int nj = 0;
  for (int si = 0; si < L.ns; ++si) {
    const StageL& g = L.st[si];
    if (g.L == 0) continue;
    const bool pack = L.bf && nj + 2 <= kMaxPackJobs && (g.C == 16 || g.C == 32 || g.C == 64);
    if (pack)
      jobs[nj++] = {params + g.off_blk, g.blk_stride, g.L, g.C, (const int32_t*)(b + g.w_src), c->gamma, b + g.wbuf,
                    g.wstride, c->param_kind != ASR_PARAM_REGULAR ? (const int32_t*)(b + g.theta_dst) : nullptr,
                    g.ntheta};
    else
      ASR_TRY(asr_theta_to_w(params + g.off_blk, g.blk_stride, g.L, g.C, (const int32_t*)(b + g.w_src), c->gamma,
                             b + g.wbuf, g.wstride, wdt, s));
    if (training && L.sep_bwd) {
      if (pack)
        jobs[nj++] = {params + g.off_blk, g.blk_stride, g.L, g.C, (const int32_t*)(b + g.w_src_bwd), 0.f,
                      b + g.wbuf_bwd, g.wstride, nullptr, 0};
      else
        ASR_TRY(asr_theta_to_w(params + g.off_blk, g.blk_stride, g.L, g.C, (const int32_t*)(b + g.w_src_bwd), 0.f,
                               b + g.wbuf_bwd, g.wstride, wdt, s));
    }
  }
  if (nj) ASR_TRY(theta_to_w_bf16_jobs(jobs, nj, s));
  ASR_TRY(stem_forward(images, c->input_u8, params + L.off_c1k, params + L.off_c1b, c->N, c->H, c->W, c->Cin,
                       c->C[0], c->subtract_mean, inv_std, c->use_norm, b + L.act0, L.bf ? 1 : 0, s));
  const void* x = b + L.act0;
  for (int si = 0; si < L.ns; ++si) {
    const StageL& g = L.st[si];
    if (g.tdirect) {  // bf16 in, bf16 out
      const float* pt = params + g.off_t;
      const long e2 = 9L * g.Cp * g.C;
      ASR_TRY(trans_fwd_lds(x, b + g.act_tb, (uint8_t*)(b + g.mask_t), pt, pt + e2, pt + e2 + g.C,
                            pt + e2 + g.C + (long)g.Cp * g.C, 1, c->N, g.Hp, g.Wp, g.Cp, g.C, s));
      x = b + g.act_tb;
    } else if (g.S) {
      const float* pt = params + g.off_t;
      const long e2 = 9L * g.Cp * g.C;
      const float* xt = (const float*)x;
      if (L.bf) {  // the transition in fp32: its input converted (and kept for the backward), its output back to bf16
        ASR_TRY(convert_bf16_f32(x, b + g.xin32, (long)c->N * g.Hp * g.Wp * g.Cp, 1, s));
        xt = (const float*)(b + g.xin32);
      }
      ASR_TRY(trans_forward(xt, (float*)(b + g.act_t), (uint8_t*)(b + g.mask_t), pt, pt + e2, pt + e2 + g.C,
                            pt + e2 + g.C + (long)g.Cp * g.C, c->N, g.Hp, g.Wp, g.Cp, g.C, g.S, s));
      x = b + g.act_t;
      if (L.bf) {
        ASR_TRY(convert_bf16_f32(b + g.act_t, b + g.act_tb, g.P, 0, s));
        x = b + g.act_tb;
      }
    }
    if (g.L == 0) continue;
    if (g.img32) {  // fp32: all L blocks in one launch, a workgroup per image
      if (x != b + g.x0)
        ASR_TRY(hip_check(hipMemcpyAsync(b + g.x0, x, (size_t)g.P * 4, hipMemcpyDeviceToDevice, s), "hipMemcpyAsync"));
      ASR_TRY(stage_img32_forward((const float*)(b + g.x0), (float*)(b + g.acts), g.P, (uint8_t*)(b + g.masks),
                                  g.mask_bytes, (const float*)(b + g.wbuf), g.wstride, params + g.off_blk + g.ntheta,
                                  g.blk_stride, c->h, c->N, g.H, g.W, g.C, g.L, s));
      x = b + g.acts + (size_t)(g.L - 1) * g.P * 4;
      continue;
    }
    if (g.img) {  // all L blocks in one launch, a workgroup per image
      if (x != b + g.x0)
        ASR_TRY(hip_check(hipMemcpyAsync(b + g.x0, x, (size_t)g.P * 2, hipMemcpyDeviceToDevice, s), "hipMemcpyAsync"));
      ASR_TRY(stage_img_forward(b + g.x0, b + g.acts, g.P, (uint8_t*)(b + g.masks), g.mask_bytes, b + g.wbuf, g.wstride,
                                params + g.off_blk + g.ntheta, g.blk_stride, c->h, c->N, g.H, g.W, g.C, g.L, s));
      x = b + g.acts + (size_t)(g.L - 1) * g.P * 2;
      continue;
    }
    if (g.deep) {  // all L blocks in one launch, images resident in LDS
      if (x != b + g.x0)
        ASR_TRY(hip_check(hipMemcpyAsync(b + g.x0, x, (size_t)g.P * 2, hipMemcpyDeviceToDevice, s), "hipMemcpyAsync"));
      ASR_TRY(deep16_forward(b + g.x0, b + g.acts, g.P, (uint8_t*)(b + g.masks), g.mask_bytes, b + g.wbuf,
                             params + g.off_blk + g.ntheta, g.blk_stride, c->h, c->N, g.L, true, s));
      x = b + g.acts + (size_t)(g.L - 1) * g.P * 2;
      continue;
    }
    for (int l = 0; l < g.L; ++l) {
      unsigned char* y = b + g.acts + (size_t)l * g.P * L.act_bytes;
      uint8_t* mk = (uint8_t*)(b + g.masks) + (size_t)l * g.mask_bytes;
      const unsigned char* wl = b + g.wbuf + (size_t)l * g.wstride * L.act_bytes;
      const float* bl = params + g.off_blk + (long)l * g.blk_stride + g.ntheta;
      if (L.bf)  // (every width on the any-width bf16 kernels: one slab-row count per stage)
        ASR_TRY(convb_forward(x, y, mk, wl, bl, c->h, c->N, g.H, g.W, g.C, s));
      else
        ASR_TRY(asr_conv_forward(ASR_MODE_EULER, x, y, mk, wl, bl, c->h, c->N, g.H, g.W, g.C, ASR_F32, s));
      x = y;
    }
  }
  *xL = x;
  return ASR_OK;
}

}  // namespace
}  // namespace asr

using namespace asr;

extern "C" {

int asr_transition_forward(const float* x, float* y, uint8_t* mask, const float* k2, const float* b2, const float* k1,
                           const float* b1, int N, int H, int W, int Ci, int Co, int stride, asr_stream_t stream) {
  ASR_TRY(check_trans(N, H, W, Ci, Co, stride));
  if (!x || !y || !k2 || !b2 || !k1 || !b1) return fail(ASR_E_ARG, "asr_transition_forward: null pointer");
  return trans_forward(x, y, mask, k2, b2, k1, b1, N, H, W, Ci, Co, stride, (hipStream_t)stream);
}

size_t asr_transition_backward_workspace_bytes(int N, int H, int W, int Ci, int Co, int stride) {
  if (check_trans(N, H, W, Ci, Co, stride) != ASR_OK) return 0;
  return trans_ws_bytes(N, H, W, Ci, Co, stride);
}

int asr_transition_backward(const float* dy, const float* x, const uint8_t* mask, const float* k2, const float* k1,
                            int N, int H, int W, int Ci, int Co, int stride, float* dx, float* dparams, void* ws,
                            size_t ws_bytes, asr_stream_t stream) {
  ASR_TRY(check_trans(N, H, W, Ci, Co, stride));
  if (!dy || !x || !mask || !k2 || !k1) return fail(ASR_E_ARG, "asr_transition_backward: null pointer");
  if (dparams && (!ws || ws_bytes < trans_ws_bytes(N, H, W, Ci, Co, stride)))
    return fail(ASR_E_WORKSPACE, "asr_transition_backward: workspace too small");
  return trans_backward(dy, x, mask, k2, k1, N, H, W, Ci, Co, stride, dx, dparams, (float*)ws, (hipStream_t)stream);
}

int asr_stages_check(const asr_stages_config* cfg) { return stages_check(cfg); }

long asr_stages_param_count(const asr_stages_config* cfg) {
  if (stages_check(cfg) != ASR_OK) return -1;
  return stages_layout(cfg).n_params;
}

size_t asr_stages_workspace_bytes(const asr_stages_config* cfg) {
  if (stages_check(cfg) != ASR_OK) return 0;
  return stages_layout(cfg).total;
}

int asr_stages_prepare(const asr_stages_config* cfg, void* ws, size_t ws_bytes) {
  ASR_TRY(stages_check(cfg));
  const SLayout L = stages_layout(cfg);
  if (!stages_layout_valid(L)) return fail(ASR_E_ARG, "asr_stages: internal workspace layout error");
  if (!ws || ws_bytes < L.total) return fail(ASR_E_WORKSPACE, "asr_stages_prepare: workspace too small");
  ASR_TRY(check_ws_device(ws, "asr_stages_prepare"));
  unsigned char* b = (unsigned char*)ws;
  for (int s = 0; s < L.ns; ++s) {
    const StageL& g = L.st[s];
    std::vector<int32_t> w_src((size_t)g.E), theta_dst((size_t)g.ntheta * 2);
    ASR_TRY(param_map(g.C, cfg->param_kind, cfg->antisymmetric, w_src.data(), theta_dst.data()));
    ASR_TRY(hip_check(hipMemcpy(b + g.w_src, w_src.data(), w_src.size() * 4, hipMemcpyHostToDevice), "hipMemcpy"));
    ASR_TRY(hip_check(hipMemcpy(b + g.theta_dst, theta_dst.data(), theta_dst.size() * 4, hipMemcpyHostToDevice),
                      "hipMemcpy"));
    if (L.sep_bwd) {
      std::vector<int32_t> w_bwd((size_t)g.E);
      ASR_TRY(param_map_transpose(g.C, w_src.data(), w_bwd.data()));
      ASR_TRY(hip_check(hipMemcpy(b + g.w_src_bwd, w_bwd.data(), w_bwd.size() * 4, hipMemcpyHostToDevice), "hipMemcpy"));
    }
  }
  return ASR_OK;
}

int asr_stages_forward(const asr_stages_config* cfg, const float* params, const void* images, float* probs, void* ws,
                       size_t ws_bytes, asr_stream_t stream) {
  ASR_TRY(stages_check(cfg));
  const SLayout L = stages_layout(cfg);
  if (!stages_layout_valid(L)) return fail(ASR_E_ARG, "asr_stages: internal workspace layout error");
  if (!params || !images || !probs) return fail(ASR_E_ARG, "asr_stages_forward: null pointer");
  if (!ws || ws_bytes < L.total) return fail(ASR_E_WORKSPACE, "asr_stages_forward: workspace too small");
  ASR_TRY(check_ws_device(ws, "asr_stages_forward"));
  hipStream_t s = (hipStream_t)stream;
  unsigned char* b = (unsigned char*)ws;
  const void* xL = nullptr;
  ASR_TRY(stages_forward_impl(cfg, L, params, images, false, b, s, &xL));
  const StageL& g = L.st[L.ns - 1];
  return head(xL, L.bf ? 1 : 0, params + L.off_fck, params + L.off_fcb, nullptr, cfg->N, g.H * g.W, g.C,
              cfg->num_classes, probs, nullptr, nullptr, nullptr, nullptr, s);
}

int asr_stages_forward_backward(const asr_stages_config* cfg, const float* params, const void* images,
                                const float* targets, float* grads, float* loss, float* probs, void* ws,
                                size_t ws_bytes, asr_stream_t stream) {
  ASR_TRY(stages_check(cfg));
  const SLayout L = stages_layout(cfg);
  if (!stages_layout_valid(L)) return fail(ASR_E_ARG, "asr_stages: internal workspace layout error");
  if (!params || !images || !targets || !grads || !loss) return fail(ASR_E_ARG, "asr_stages_forward_backward: null");
  if (!ws || ws_bytes < L.total) return fail(ASR_E_WORKSPACE, "asr_stages_forward_backward: workspace too small");
  ASR_TRY(check_ws_device(ws, "asr_stages_forward_backward"));
  hipStream_t s = (hipStream_t)stream;
  unsigned char* b = (unsigned char*)ws;
  const int N = cfg->N, K = cfg->num_classes;
  const size_t ab = L.act_bytes;
  const void* xL = nullptr;
  ASR_TRY(stages_forward_impl(cfg, L, params, images, true, b, s, &xL));
  // the chain gradient ping-pongs between dA and dB (bf16 nets: bf16 through the blocks)
  unsigned char* d = b + L.dA;
  unsigned char* e = b + L.dB;
  const StageL& top = L.st[L.ns - 1];
  ASR_TRY(head(xL, L.bf ? 1 : 0, params + L.off_fck, params + L.off_fcb, targets, N, top.H * top.W, top.C, K,
               probs ? probs : (float*)(b + L.probs), (float*)(b + L.loss_per), (float*)(b + L.dlogits),
               (float*)(b + L.gap), d, s));
  ASR_TRY(head_param_grads((const float*)(b + L.gap), (const float*)(b + L.dlogits), N, top.C, K, grads + L.off_fck,
                           grads + L.off_fcb, (const float*)(b + L.loss_per), loss, s));
  for (int si = L.ns - 1; si >= 0; --si) {
    const StageL& g = L.st[si];
    // the stage's chain input: its transition's output, else the previous stage's last activation
    // (in the net's activation type; a bf16 net's transition input is also kept in fp32, xin32)
    const unsigned char* prev_out = b + L.act0;
    for (int sp = si - 1; sp >= 0; --sp) {
      const StageL& q = L.st[sp];
      if (q.L > 0) { prev_out = b + q.acts + (size_t)(q.L - 1) * q.P * ab; break; }
      if (q.S) { prev_out = b + (L.bf ? q.act_tb : q.act_t); break; }
    }
    const unsigned char* chain_in = g.S ? b + (L.bf ? g.act_tb : g.act_t) : prev_out;
    const float gam = L.sep_bwd ? 0.f : cfg->gamma;
    int nsl = 0;
    if (g.deep) {  // all L blocks in one launch (dx resident in LDS), one slab set per layer
      int rows = 0, in_b = 0;
      ASR_TRY(deep16_backward(d, e, b + g.x0, g.P, (const uint8_t*)(b + g.masks), g.mask_bytes,
                              b + (L.sep_bwd ? g.wbuf_bwd : g.wbuf), cfg->h, 2.f * gam, N, g.L,
                              (float*)(b + g.slabs), &rows, &in_b, s));
      if (rows != g.slab_rows) return fail(ASR_E_WORKSPACE, "asr_stages: deep16 slab rows %d != %d", rows, g.slab_rows);
      if (in_b) std::swap(d, e);
      ASR_TRY(reduce_slabs_to_groups((const float*)(b + g.slabs), g.L * rows, g.E + g.C, (float*)(b + g.grp), s));
      ASR_TRY(project_layers((float*)(b + g.grp), g.grp_stride, reduce_groups(rows), g.E, g.C,
                             (const int32_t*)(b + g.theta_dst), g.ntheta, g.L, grads + g.off_blk, g.blk_stride, s));
    }
    if (g.img) {  // input gradients in one launch; then each layer's weight gradient from its stored input gradient
      ASR_TRY(stage_img_backward(d, b + g.dys, g.P, e, (const uint8_t*)(b + g.masks), g.mask_bytes,
                                 b + (L.sep_bwd ? g.wbuf_bwd : g.wbuf), g.wstride, cfg->h, 2.f * gam, N, g.H, g.W, g.C,
                                 g.L, s));
      // every layer's weight gradient in one launch: x_l = x0 + l P, its input gradient dys + l P
      ASR_TRY(wgradb_layers(b + g.x0, g.P, b + g.dys, g.P, (const uint8_t*)(b + g.masks), g.mask_bytes, cfg->h, N, g.H,
                            g.W, g.C, g.L, (float*)(b + g.slabs), g.slab_stride, &nsl, s));
      if (nsl > g.slab_rows) return fail(ASR_E_WORKSPACE, "asr_stages: %d slab rows > the workspace's %d", nsl, g.slab_rows);
      std::swap(d, e);
    }
    if (g.img32) {  // fp32: input gradients in one launch, every layer's weight gradient in one launch
      ASR_TRY(stage_img32_backward((const float*)d, (float*)(b + g.dys), g.P, (float*)e, (const uint8_t*)(b + g.masks),
                                   g.mask_bytes, (const float*)(b + (L.sep_bwd ? g.wbuf_bwd : g.wbuf)), g.wstride,
                                   cfg->h, 2.f * gam, N, g.H, g.W, g.C, g.L, s));
      ASR_TRY(wgrad32_layers((const float*)(b + g.x0), g.P, (const float*)(b + g.dys), g.P, (const uint8_t*)(b + g.masks),
                             g.mask_bytes, cfg->h, N, g.H, g.W, g.C, g.L, (float*)(b + g.slabs), g.slab_stride, &nsl, s));
      if (nsl > g.slab_rows) return fail(ASR_E_WORKSPACE, "asr_stages: %d slab rows > the workspace's %d", nsl, g.slab_rows);
      std::swap(d, e);
    }
    for (int l = (g.deep || g.img || g.img32) ? -1 : g.L - 1; l >= 0; --l) {
      const unsigned char* x_in = l == 0 ? chain_in : b + g.acts + (size_t)(l - 1) * g.P * ab;
      const unsigned char* wl = b + (L.sep_bwd ? g.wbuf_bwd : g.wbuf) + (size_t)l * g.wstride * ab;
      const uint8_t* mk = (const uint8_t*)(b + g.masks) + (size_t)l * g.mask_bytes;
      float* sl = (float*)(b + g.slabs) + (size_t)l * g.slab_stride;
      // the block's weight-gradient slabs stay in its own slot: the stage's blocks are reduced
      // (pass 1, one launch) and projected (pass 2 + projection, one launch) after the loop
      if (L.bf)
        ASR_TRY(convb_backward(d, mk, x_in, wl, cfg->h, 2.f * gam, N, g.H, g.W, g.C, e, true, sl, &nsl, s));
      else
        ASR_TRY(conv_backward_keep_slabs(d, x_in, mk, wl, cfg->h, gam, N, g.H, g.W, g.C, e, b + L.cws, sl, &nsl, s));
      if (nsl > g.slab_rows)  // (the device differs from the one the workspace was sized on)
        return fail(ASR_E_WORKSPACE, "asr_stages: %d slab rows > the workspace's %d (sized on another device?)", nsl,
                    g.slab_rows);
      std::swap(d, e);
    }
    if (g.L > 0 && !g.deep)
      ASR_TRY(reduce_slab_layers((const float*)(b + g.slabs), g.slab_stride, nsl, g.E + g.C, (float*)(b + g.grp),
                                 g.grp_stride, g.L, s));
    if (g.L > 0 && !g.deep)
      ASR_TRY(project_layers((float*)(b + g.grp), g.grp_stride, reduce_groups(nsl), g.E, g.C,
                             (const int32_t*)(b + g.theta_dst), g.ntheta, g.L, grads + g.off_blk, g.blk_stride, s));
    if (g.S) {
      const float* pt = params + g.off_t;
      const long e2 = 9L * g.Cp * g.C;
      const long Pin = (long)N * g.Hp * g.Wp * g.Cp;
      if (g.tdirect) {
        ASR_TRY(trans_backward_bf16((const bf16*)d, (const bf16*)prev_out, (const uint8_t*)(b + g.mask_t), pt,
                                    pt + e2 + g.C, N, g.Hp, g.Wp, g.Cp, g.C, g.S, (bf16*)e, grads + g.off_t,
                                    (float*)(b + L.tws), s));
      } else if (L.bf) {  // in fp32: dy converted up, the transition's kept fp32 input, dx converted back down
        float* dy32 = (float*)(b + L.t32a);
        float* dx32 = (float*)(b + L.t32b);
        ASR_TRY(convert_bf16_f32(d, dy32, g.P, 1, s));
        ASR_TRY(trans_backward(dy32, (const float*)(b + g.xin32), (const uint8_t*)(b + g.mask_t), pt, pt + e2 + g.C,
                               N, g.Hp, g.Wp, g.Cp, g.C, g.S, dx32, grads + g.off_t, (float*)(b + L.tws), s));
        ASR_TRY(convert_bf16_f32(dx32, e, Pin, 0, s));
      } else {
        ASR_TRY(trans_backward((const float*)d, (const float*)prev_out, (const uint8_t*)(b + g.mask_t), pt,
                               pt + e2 + g.C, N, g.Hp, g.Wp, g.Cp, g.C, g.S, (float*)e, grads + g.off_t,
                               (float*)(b + L.tws), s));
      }
      std::swap(d, e);
    }
  }
  // stem: conv1 kernel / bias gradients from dz1 = dx1 [x1 > 0].  bf16 nets at C = 16 / 64: dz1 in place
  // (k_relu_grad_bf16), then the weight gradient on MFMA (k_stem_wgrad_mfma: bf16 (v - mean) and dz1,
  // exact products for u8 images with a half-integer mean, fp32 sums; 51 -> ~18 us at he32_bf16's batch);
  // else the fp32 VALU kernel, which applies the relu' itself
  const float inv_std = cfg->use_norm ? 1.f / cfg->divide_by_stddev : 1.f;
  int nsl = 0;
  const long P0 = (long)N * cfg->H * cfg->W * cfg->C[0];
  if (L.bf && P0 % 8 == 0 && stem_wgrad_mfma_supported(cfg->Cin, cfg->H, cfg->W, cfg->C[0])) {
    ASR_TRY(relu_grad_bf16(d, b + L.act0, P0, s));
    ASR_TRY(stem_wgrad_mfma(images, cfg->input_u8, d, N, cfg->H, cfg->W, cfg->Cin, cfg->C[0], cfg->subtract_mean,
                            inv_std, cfg->use_norm, (float*)(b + L.sslabs), &nsl, s));
  } else {
    ASR_TRY(stem_wgrad(images, cfg->input_u8, d, b + L.act0, L.bf ? 1 : 0, N, cfg->H, cfg->W, cfg->Cin, cfg->C[0],
                       cfg->subtract_mean, inv_std, cfg->use_norm, (float*)(b + L.sslabs), &nsl, s));
  }
  if (nsl > kMaxStemSlabs) return fail(ASR_E_UNSUPPORTED, "asr_stages: stem slabs %d > %d", nsl, kMaxStemSlabs);
  return reduce_and_project((const float*)(b + L.sslabs), nsl, 9L * cfg->Cin * cfg->C[0], cfg->C[0], nullptr, 0,
                            nullptr, grads + L.off_c1b, grads + L.off_c1k, (float*)(b + L.sred), s);
}

}  // extern "C"
