// Stem (input normalisation + conv1 + relu) and head (GAP + Dense + softmax +
// Keras cross-entropy) of the single-block ResNet, forward and backward.
//
// Reference: models/tfkeras_resnets.py:555-559 (Lambda x-127.5, x/127.5),
// :563-572 (conv1: regular 3x3 SAME conv, filters_per_block[0], relu),
// :595-597 (GlobalAveragePooling2D, Dense(num_classes, softmax) 'fc');
// training/training.py:295 (mean Keras categorical cross-entropy on the
// probabilities).  These are small next to the L Euler blocks; each is one
// image per workgroup with the image staged (normalised, zero-padded) in LDS.
#include <math.h>

#include "asr_common.h"


namespace asr {

// LDS image: (H+2) x (W+2) x CIN floats, normalised, zero halo.  The halo
// is written once (zero_tile_halo); stage_image fills the interior from
// 16-byte vector loads, all of a thread's loads issued before their use (one
// image per workgroup: a latency-serialised element loop dominated the stem).
template <int CIN>
__device__ __forceinline__ void zero_tile(float* tile, int H, int W) {
  for (int i = threadIdx.x; i < (H + 2) * (W + 2) * CIN; i += blockDim.x) tile[i] = 0.f;
}

template <int CIN, typename Tin>
__device__ __forceinline__ void stage_image(const Tin* __restrict__ img, float* tile, int H, int W, float mean,
                                            float inv_std, int use_norm) {
  constexpr int EPV = 16 / sizeof(Tin);  // elements per 16-B vector
  constexpr int KV = 4;                  // vectors in flight per thread
  const int TW = W + 2, nel = H * W * CIN;
  const bool vec_ok = ((uintptr_t)img % 16 == 0);  // images of a 16-B multiple (e.g. 32x32x3 u8) stay aligned
  const int nvec = vec_ok ? nel / EPV : 0;
  for (int v0 = threadIdx.x; v0 < nvec; v0 += KV * blockDim.x) {
    uint4 r[KV];
#pragma unroll
    for (int k = 0; k < KV; ++k) {
      const int vi = v0 + k * blockDim.x;
      r[k] = vi < nvec ? *(const uint4*)(img + (long)vi * EPV) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < KV; ++k) {
      const int vi = v0 + k * blockDim.x;
      if (vi >= nvec) continue;
      const Tin* e = (const Tin*)&r[k];
#pragma unroll
      for (int j = 0; j < EPV; ++j) {
        const int o = vi * EPV + j, c = o % CIN, pix = o / CIN;
        float v = (float)e[j];
        if (use_norm) v = (v - mean) * inv_std;
        tile[((pix / W + 1) * TW + pix % W + 1) * CIN + c] = v;
      }
    }
  }
  for (int o = nvec * EPV + threadIdx.x; o < nel; o += blockDim.x) {  // tail (nel % EPV)
    const int c = o % CIN, pix = o / CIN;
    float v = (float)img[o];
    if (use_norm) v = (v - mean) * inv_std;
    tile[((pix / W + 1) * TW + pix % W + 1) * CIN + c] = v;
  }
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// conv1 forward: out = relu(conv3x3(norm(img)) + b); one image per block
// iteration; thread = (VEC-channel group, pixel lane) with its 9*CIN*VEC
// weights in registers, the normalised image tile in LDS.  Channel pairs
// are accumulated with packed FMAs (v_pk_fma_f32: two fp32 FMAs per lane,
// bitwise the fmaf chain of the scalar form).
template <int CIN, typename Tin, typename Tout, int VEC>
__global__ __launch_bounds__(256) void k_stem_fwd(const Tin* __restrict__ img, const float* __restrict__ w1,
                                                  const float* __restrict__ b1, int N, int H, int W, int C,
                                                  float mean, float inv_std, int use_norm, Tout* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* tile = sm;  // (H+2)(W+2)CIN
  constexpr int VP = (VEC + 1) / 2;  // channel pairs
  const int NG = C / VEC, PLN = max(1, 256 / NG);
  const int cg = threadIdx.x % NG, pl = threadIdx.x / NG;
  const bool active = threadIdx.x < PLN * NG;
  f32x2 wr[9 * CIN][VP], bz[VP];
#pragma unroll
  for (int k = 0; k < 9 * CIN; ++k)
#pragma unroll
    for (int v = 0; v < VP; ++v)
      wr[k][v] = f32x2{active ? w1[k * C + cg * VEC + 2 * v] : 0.f,
                       (active && 2 * v + 1 < VEC) ? w1[k * C + cg * VEC + 2 * v + 1] : 0.f};
#pragma unroll
  for (int v = 0; v < VP; ++v)
    bz[v] = f32x2{(active && b1) ? b1[cg * VEC + 2 * v] : 0.f,
                  (active && b1 && 2 * v + 1 < VEC) ? b1[cg * VEC + 2 * v + 1] : 0.f};
  const int TW = W + 2;
  zero_tile<CIN>(tile, H, W);
  for (int n = blockIdx.x; n < N; n += gridDim.x) {
    __syncthreads();
    stage_image<CIN>(img + (long)n * H * W * CIN, tile, H, W, mean, inv_std, use_norm);
    __syncthreads();
    if (!active) continue;
    for (int p = pl; p < H * W; p += PLN) {
      const int x = p % W, y = p / W;
      f32x2 acc[VP];
#pragma unroll
      for (int v = 0; v < VP; ++v) acc[v] = bz[v];
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const float* tp = tile + ((y + tap / 3) * TW + x + tap % 3) * CIN;
#pragma unroll
        for (int ci = 0; ci < CIN; ++ci) {
          const float xv = tp[ci];
#pragma unroll
          for (int v = 0; v < VP; ++v) acc[v] = __builtin_elementwise_fma(f32x2{xv, xv}, wr[tap * CIN + ci][v], acc[v]);
        }
      }
      Tout* o = out + ((long)n * H * W + p) * C + cg * VEC;
      if constexpr (VEC == 4 && sizeof(Tout) == 2) {
        bf16x4 r;
#pragma unroll
        for (int v = 0; v < 4; ++v) r[v] = (bf16)fmaxf(acc[v / 2][v % 2], 0.f);
        *(bf16x4*)o = r;
      } else {
#pragma unroll
        for (int v = 0; v < VEC; ++v) o[v] = from_f32<Tout>(fmaxf(acc[v / 2][v % 2], 0.f));
      }
    }
  }
}

// conv1 weight gradient: dz1 = dx1 * [x1 > 0]; slab[blk] = [dW1 (9*CIN*C) | db1 (C)].
// Thread = (4-channel group cg, pixel lane); the normalised image tile in
// LDS, one broadcast LDS read per tap feeds 4 channels (packed FMAs).  The
// pixel lanes of a wave reduce by shuffles, the 4 waves through LDS (fixed
// order: deterministic).  C % 4 == 0 and C <= 64.
template <int CIN, typename Tin, typename T>
__global__ __launch_bounds__(256) void k_stem_wgrad(const Tin* __restrict__ img, const T* __restrict__ dx1,
                                                    const T* __restrict__ x1, int N, int H, int W, int C, float mean,
                                                    float inv_std, int use_norm, float* __restrict__ slabs) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  constexpr int KC = 9 * CIN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int NG = C / 4;     // channel groups (<= 16)
  const int PL = 256 / NG;  // pixel lanes
  const int cg = tid % NG, pl = tid / NG;
  f32x2 acc[KC + 1][2];
#pragma unroll
  for (int k = 0; k <= KC; ++k) acc[k][0] = acc[k][1] = f32x2{0.f, 0.f};
  float* tile = sm;
  const int TW = W + 2;
  zero_tile<CIN>(tile, H, W);
  for (int n = blockIdx.x; n < N; n += gridDim.x) {
    __syncthreads();
    stage_image<CIN>(img + (long)n * H * W * CIN, tile, H, W, mean, inv_std, use_norm);
    __syncthreads();
    const T* d = dx1 + (long)n * H * W * C + cg * 4;
    const T* a = x1 + (long)n * H * W * C + cg * 4;
    constexpr int U = 4;  // pixels per batch: all global loads issued before use
    for (int p0 = pl; p0 < H * W; p0 += U * PL) {
      f32x2 gv[U][2];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int p = p0 + u * PL;
        const int pc = p < H * W ? p : 0;
        float dv[4], av[4];
        if constexpr (sizeof(T) == 2) {
          const bf16x4 d4 = *(const bf16x4*)(d + (long)pc * C), a4 = *(const bf16x4*)(a + (long)pc * C);
#pragma unroll
          for (int v = 0; v < 4; ++v) dv[v] = (float)d4[v], av[v] = (float)a4[v];
        } else {
          const float4 d4 = *(const float4*)(d + (long)pc * C), a4 = *(const float4*)(a + (long)pc * C);
          dv[0] = d4.x, dv[1] = d4.y, dv[2] = d4.z, dv[3] = d4.w;
          av[0] = a4.x, av[1] = a4.y, av[2] = a4.z, av[3] = a4.w;
        }
        float g4[4];
#pragma unroll
        for (int v = 0; v < 4; ++v) g4[v] = (p < H * W && av[v] > 0.f) ? dv[v] : 0.f;
        gv[u][0] = f32x2{g4[0], g4[1]};
        gv[u][1] = f32x2{g4[2], g4[3]};
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int p = p0 + u * PL;
        const int pc = p < H * W ? p : 0;
        const int x = pc % W, y = pc / W;
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
          const float* tp = tile + ((y + tap / 3) * TW + x + tap % 3) * CIN;
#pragma unroll
          for (int ci = 0; ci < CIN; ++ci) {
            const float xv = tp[ci];
#pragma unroll
            for (int h = 0; h < 2; ++h)
              acc[tap * CIN + ci][h] = __builtin_elementwise_fma(f32x2{xv, xv}, gv[u][h], acc[tap * CIN + ci][h]);
          }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) acc[KC][h] += gv[u][h];
      }
    }
  }
  // pixel lanes of this wave: lanes cg, cg+NG, ... (NG divides 64)
#pragma unroll
  for (int k = 0; k <= KC; ++k)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        float v = acc[k][h][e];
        for (int off = NG; off < 64; off <<= 1) v += __shfl_xor(v, off);
        acc[k][h][e] = v;
      }
  __syncthreads();
  float* red = sm;  // [4 waves][KC+1][C]
  if (lane < NG)
#pragma unroll
    for (int k = 0; k <= KC; ++k)
#pragma unroll
      for (int v = 0; v < 4; ++v) red[((long)wave * (KC + 1) + k) * C + cg * 4 + v] = acc[k][v / 2][v % 2];
  __syncthreads();
  float* slab = slabs + (long)blockIdx.x * (KC * C + C);
  for (int i = tid; i < (KC + 1) * C; i += blockDim.x) {
    const long st = (long)(KC + 1) * C;
    slab[i] = (red[i] + red[st + i]) + (red[2 * st + i] + red[3 * st + i]);  // i = k*C + o
  }
}

// GAP -> Dense(K) -> softmax [-> Keras CE loss and its gradient] per image.
// (TF 1.12 keras.backend.categorical_crossentropy: renormalise, clip
// [1e-7, 1-1e-7], -sum t*log q; the clip gradient passes on the closed
// interval.)  dxL[n,p,c] = (dlogits . fc[c,:]) / (H*W) for every pixel; or,
// with growL, only that per-(image, channel) row (the GAP gradient is
// constant over the pixels, models/tfkeras_resnets.py:595-597): the C=64
// stacked backward stages its top block's dy from it instead of reading a
// full tensor.
template <typename T, int VEC>
__global__ __launch_bounds__(256) void k_head(const T* __restrict__ xL, const float* __restrict__ fck,
                                              const float* __restrict__ fcb, const float* __restrict__ targets,
                                              int HW, int C, int K, float inv_n, float* __restrict__ probs,
                                              float* __restrict__ loss_per, float* __restrict__ dlogits,
                                              float* __restrict__ gap, T* __restrict__ dxL, T* __restrict__ growL) {
  __shared__ float red[256 * VEC];
  __shared__ float gs[256];
  __shared__ float lg[256];
  __shared__ float dl[256];
  const int n = blockIdx.x, tid = threadIdx.x;
  const int NQ = C / VEC;
  const int PL = max(1, 256 / NQ);
  const int q = tid % NQ, pl = tid / NQ;
  float s[VEC];
#pragma unroll
  for (int v = 0; v < VEC; ++v) s[v] = 0.f;
  if (pl < PL && tid < PL * NQ) {
    const T* base = xL + (long)n * HW * C + q * VEC;
    // 8 independent loads in flight per thread: at 2 blocks per CU the read
    // is latency-bound otherwise
#pragma unroll 8
    for (int p = pl; p < HW; p += PL) {
      if constexpr (VEC == 8 && sizeof(T) == 2) {
        const bf16x8 v8 = *(const bf16x8*)(base + (long)p * C);
#pragma unroll
        for (int v = 0; v < 8; ++v) s[v] += (float)v8[v];
      } else if constexpr (VEC == 4 && sizeof(T) == 4) {
        const float4 v4 = *(const float4*)(base + (long)p * C);
        s[0] += v4.x;
        s[1] += v4.y;
        s[2] += v4.z;
        s[3] += v4.w;
      } else {
#pragma unroll
        for (int v = 0; v < VEC; ++v) s[v] += to_f32(base[(long)p * C + v]);
      }
    }
  }
#pragma unroll
  for (int v = 0; v < VEC; ++v) red[tid * VEC + v] = s[v];
  __syncthreads();
  if (tid < C) {
    const int qq = tid / VEC, v = tid % VEC;
    float t = 0.f;
    for (int p = 0; p < PL; ++p) t += red[(p * NQ + qq) * VEC + v];
    t /= (float)HW;
    gs[tid] = t;
    if (gap) gap[(long)n * C + tid] = t;
  }
  __syncthreads();
  if (tid < K) {
    float a = fcb ? fcb[tid] : 0.f;
    for (int c = 0; c < C; ++c) a = fmaf(gs[c], fck[(long)c * K + tid], a);
    lg[tid] = a;
  }
  __syncthreads();
  if (tid == 0) {
    float m = -INFINITY;
    for (int k = 0; k < K; ++k) m = fmaxf(m, lg[k]);
    float S = 0.f;
    for (int k = 0; k < K; ++k) {
      const float e = expf(lg[k] - m);
      lg[k] = e;
      S += e;
    }
    float s2 = 0.f;
    for (int k = 0; k < K; ++k) {
      lg[k] /= S;
      s2 += lg[k];
      if (probs) probs[(long)n * K + k] = lg[k];
    }
    if (targets) {
      const float eps = 1e-7f;
      float loss = 0.f, sdq_p = 0.f;
      for (int k = 0; k < K; ++k) {
        const float qv = lg[k] / s2;
        const float qc = fminf(fmaxf(qv, eps), 1.f - eps);
        const float t = targets[(long)n * K + k];
        loss -= t * logf(qc);
        const float dq = (qv >= eps && qv <= 1.f - eps) ? -t / qc * inv_n : 0.f;
        dl[k] = dq;
        sdq_p += dq * lg[k];
      }
      if (loss_per) loss_per[n] = loss;
      float sp_dp = 0.f;
      for (int k = 0; k < K; ++k) {
        const float dp = dl[k] / s2 - sdq_p / (s2 * s2);
        dl[k] = dp;
        sp_dp += lg[k] * dp;
      }
      for (int k = 0; k < K; ++k) {
        const float d = lg[k] * (dl[k] - sp_dp);
        dl[k] = d;
        if (dlogits) dlogits[(long)n * K + k] = d;
      }
    }
  }
  __syncthreads();
  if (targets && growL) {
    if (tid < C) {
      float a = 0.f;
      for (int k = 0; k < K; ++k) a = fmaf(dl[k], fck[(long)tid * K + k], a);
      growL[(long)n * C + tid] = from_f32<T>(a / (float)HW);
    }
  } else if (targets && dxL) {
    if (tid < C) {
      float a = 0.f;
      for (int k = 0; k < K; ++k) a = fmaf(dl[k], fck[(long)tid * K + k], a);
      gs[tid] = a / (float)HW;
    }
    __syncthreads();
    T* o = dxL + (long)n * HW * C;
    for (long i = tid; i < (long)HW * NQ; i += 256) {
      const int qq = (int)(i % NQ);
      T* dst = o + i * VEC;
      if constexpr (VEC == 8 && sizeof(T) == 2) {
        bf16x8 r;
#pragma unroll
        for (int v = 0; v < 8; ++v) r[v] = (bf16)gs[qq * 8 + v];
        *(bf16x8*)dst = r;
      } else {
#pragma unroll
        for (int v = 0; v < VEC; ++v) dst[v] = from_f32<T>(gs[qq * VEC + v]);
      }
    }
  }
}

// Dense parameter gradients and the batch-mean loss.  Block c < C:
// dfck[c][k] = sum_n gap[n][c] dl[n][k];  block C: dfcb, mean loss.
__global__ __launch_bounds__(256) void k_head_param_grads(const float* __restrict__ gap,
                                                          const float* __restrict__ dlogits, int N, int C, int K,
                                                          float* __restrict__ dfck, float* __restrict__ dfcb,
                                                          const float* __restrict__ loss_per,
                                                          float* __restrict__ loss_out) {
  __shared__ float red[256];
  const int tid = threadIdx.x, c = blockIdx.x;
  const int NL = max(1, 256 / K);
  const int k = tid % K, nl = tid / K;
  float a = 0.f;
  if (nl < NL && tid < NL * K) {
    for (int n = nl; n < N; n += NL) {
      const float d = dlogits[(long)n * K + k];
      a = (c < C) ? fmaf(gap[(long)n * C + c], d, a) : a + d;
    }
  }
  red[tid] = a;
  __syncthreads();
  if (tid < K) {
    float s = 0.f;
    for (int g = 0; g < NL; ++g) s += red[g * K + tid];
    if (c < C)
      dfck[(long)c * K + tid] = s;
    else
      dfcb[tid] = s;
  }
  if (c == C) {
    __syncthreads();
    float l = 0.f;
    for (int n = tid; n < N; n += 256) l += loss_per[n];
    red[tid] = l;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
      if (tid < w) red[tid] += red[tid + w];
      __syncthreads();
    }
    if (tid == 0) *loss_out = red[0] / (float)N;
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
constexpr int kMaxSlabsStem = 512;

bool stem_supported(int Cin, int H, int W, int C) {
  const size_t lds = (size_t)(H + 2) * (W + 2) * Cin * 4;
  const size_t red = (size_t)4 * (9 * Cin + 1) * C * 4;
  return (Cin == 1 || Cin == 3) && C % 4 == 0 && C <= 64 && lds <= 64 * 1024 && red <= 64 * 1024;
}

static int stem_grid(int N) { return std::max(1, std::min(N, kMaxSlabsStem)); }

template <int CIN, typename Tin, typename Tout>
static void launch_stem_fwd(const void* img, const float* w1, const float* b1, int N, int H, int W, int C, float mean,
                            float inv_std, int use_norm, void* out, hipStream_t s) {
  const size_t lds = (size_t)(H + 2) * (W + 2) * CIN * 4;
  if (C % 4 == 0)
    hipLaunchKernelGGL((k_stem_fwd<CIN, Tin, Tout, 4>), dim3(stem_grid(N)), dim3(256), lds, s, (const Tin*)img, w1,
                       b1, N, H, W, C, mean, inv_std, use_norm, (Tout*)out);
  else
    hipLaunchKernelGGL((k_stem_fwd<CIN, Tin, Tout, 1>), dim3(stem_grid(N)), dim3(256), lds, s, (const Tin*)img, w1,
                       b1, N, H, W, C, mean, inv_std, use_norm, (Tout*)out);
}

int stem_forward(const void* img, int input_u8, const float* w1, const float* b1, int N, int H, int W, int Cin, int C,
                 float mean, float inv_std, int use_norm, void* out, int out_bf16, hipStream_t s) {
  if (!stem_supported(Cin, H, W, C)) return fail(ASR_E_UNSUPPORTED, "stem: unsupported shape");
#define ASR_STEM_F(CI, TI, TO) launch_stem_fwd<CI, TI, TO>(img, w1, b1, N, H, W, C, mean, inv_std, use_norm, out, s)
  if (Cin == 3) {
    if (input_u8) { if (out_bf16) ASR_STEM_F(3, uint8_t, bf16); else ASR_STEM_F(3, uint8_t, float); }
    else { if (out_bf16) ASR_STEM_F(3, float, bf16); else ASR_STEM_F(3, float, float); }
  } else {
    if (input_u8) { if (out_bf16) ASR_STEM_F(1, uint8_t, bf16); else ASR_STEM_F(1, uint8_t, float); }
    else { if (out_bf16) ASR_STEM_F(1, float, bf16); else ASR_STEM_F(1, float, float); }
  }
#undef ASR_STEM_F
  ASR_LAUNCH_CHECK("k_stem_fwd");
  return ASR_OK;
}

int stem_wgrad(const void* img, int input_u8, const void* dx1, const void* x1, int act_bf16, int N, int H, int W,
               int Cin, int C, float mean, float inv_std, int use_norm, float* slabs, int* nslabs, hipStream_t s) {
  if (!stem_supported(Cin, H, W, C)) return fail(ASR_E_UNSUPPORTED, "stem: unsupported shape");
  const int grid = stem_grid(N);
  *nslabs = grid;
  const size_t lds = std::max((size_t)(H + 2) * (W + 2) * Cin * 4, (size_t)4 * (9 * Cin + 1) * C * 4);
#define ASR_STEM_W(CI, TI, T)                                                                                   \
  hipLaunchKernelGGL((k_stem_wgrad<CI, TI, T>), dim3(grid), dim3(256), lds, s, (const TI*)img, (const T*)dx1, \
                     (const T*)x1, N, H, W, C, mean, inv_std, use_norm, slabs)
  if (Cin == 3) {
    if (input_u8) { if (act_bf16) ASR_STEM_W(3, uint8_t, bf16); else ASR_STEM_W(3, uint8_t, float); }
    else { if (act_bf16) ASR_STEM_W(3, float, bf16); else ASR_STEM_W(3, float, float); }
  } else {
    if (input_u8) { if (act_bf16) ASR_STEM_W(1, uint8_t, bf16); else ASR_STEM_W(1, uint8_t, float); }
    else { if (act_bf16) ASR_STEM_W(1, float, bf16); else ASR_STEM_W(1, float, float); }
  }
#undef ASR_STEM_W
  ASR_LAUNCH_CHECK("k_stem_wgrad");
  return ASR_OK;
}

int head(const void* xL, int act_bf16, const float* fck, const float* fcb, const float* targets, int N, int HW, int C,
         int K, float* probs, float* loss_per, float* dlogits, float* gap, void* dxL, hipStream_t s, void* growL) {
  if (C > 256 || K > 256) return fail(ASR_E_UNSUPPORTED, "head: C and num_classes must be <= 256");
  const float inv_n = 1.f / (float)N;
  if (act_bf16) {
    if (C % 8 == 0)
      hipLaunchKernelGGL((k_head<bf16, 8>), dim3(N), dim3(256), 0, s, (const bf16*)xL, fck, fcb, targets, HW, C, K,
                         inv_n, probs, loss_per, dlogits, gap, (bf16*)dxL, (bf16*)growL);
    else
      hipLaunchKernelGGL((k_head<bf16, 1>), dim3(N), dim3(256), 0, s, (const bf16*)xL, fck, fcb, targets, HW, C, K,
                         inv_n, probs, loss_per, dlogits, gap, (bf16*)dxL, (bf16*)growL);
  } else {
    if (C % 4 == 0)
      hipLaunchKernelGGL((k_head<float, 4>), dim3(N), dim3(256), 0, s, (const float*)xL, fck, fcb, targets, HW, C,
                         K, inv_n, probs, loss_per, dlogits, gap, (float*)dxL, (float*)growL);
    else
      hipLaunchKernelGGL((k_head<float, 1>), dim3(N), dim3(256), 0, s, (const float*)xL, fck, fcb, targets, HW, C,
                         K, inv_n, probs, loss_per, dlogits, gap, (float*)dxL, (float*)growL);
  }
  ASR_LAUNCH_CHECK("k_head");
  return ASR_OK;
}

int head_param_grads(const float* gap, const float* dlogits, int N, int C, int K, float* dfck, float* dfcb,
                     const float* loss_per, float* loss_out, hipStream_t s) {
  hipLaunchKernelGGL(k_head_param_grads, dim3(C + 1), dim3(256), 0, s, gap, dlogits, N, C, K, dfck, dfcb, loss_per,
                     loss_out);
  ASR_LAUNCH_CHECK("k_head_param_grads");
  return ASR_OK;
}

}  // namespace asr
