// fp32 path of the 3x3 conv / Euler block: exact fp32 FMA chains on the VALU.
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
// a zeroed buffer because C need not be a multiple of 8 here.
template <typename Tin, typename Tout, int MODE>
__global__ __launch_bounds__(256) void k_conv_f32(const Tin* __restrict__ xin, Tout* __restrict__ out,
                                                  uint32_t* __restrict__ mask, const float* __restrict__ w,
                                                  const float* __restrict__ bias, float h, float two_gamma,
                                                  const float* __restrict__ dy, const float* __restrict__ extra,
                                                  int N, int H, int W, int Ci, int Co) {
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
    for (int tap = 0; tap < 9; ++tap) {
      const int gy = y + tap / 3 - 1, gx = px + tap % 3 - 1;
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
                                                   float* __restrict__ slabs) {
  const long E = 9L * Ci * Co;
  const long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (e >= E) return;
  const int o = (int)(e % Co);
  const int i = (int)((e / Co) % Ci);
  const int tap = (int)(e / ((long)Ci * Co));
  const int sy = tap / 3 - 1, sx = tap % 3 - 1;
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

template <typename Tin, typename Tout, int MODE>
static int launch_conv_f32(const void* xin, void* out, uint8_t* mask, const float* w, const float* bias, float h,
                           float two_gamma, const float* dy, const float* extra, int N, int H, int W, int Ci, int Co,
                           hipStream_t s) {
  const long tasks = (long)N * H * ((W + 15) / 16) * ((Co + 15) / 16);
  const long blocks = (tasks + 3) / 4;
  if (blocks > 0x7fffffffL) return fail(ASR_E_ARG, "conv f32: problem too large");
  if (MODE == F_EULER && mask) {
    const long bytes = ((long)N * H * W * Co + 31) / 32 * 4;
    ASR_TRY(hip_check(hipMemsetAsync(mask, 0, bytes, s), "hipMemsetAsync(mask)"));
  }
  hipLaunchKernelGGL((k_conv_f32<Tin, Tout, MODE>), dim3((unsigned)blocks), dim3(256), 0, s, (const Tin*)xin,
                     (Tout*)out, (uint32_t*)mask, w, bias, h, two_gamma, dy, extra, N, H, W, Ci, Co);
  ASR_LAUNCH_CHECK("k_conv_f32");
  return ASR_OK;
}

int conv_f32(int fmode, const void* xin, void* out, uint8_t* mask, const float* w, const float* bias, float h,
             float two_gamma, const float* dy, int N, int H, int W, int Ci, int Co, int out_bf16, hipStream_t s,
             const float* extra) {
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

// number of row chunks used by the fp32 wgrad (bounded by kMaxSlabs in the
// workspace sizing of the callers)
int wgrad_f32_chunks(int N, int H) {
  const long R = (long)N * H;
  long chunks = std::min<long>(R, 256);
  return (int)std::max<long>(chunks, 1);
}

int wgrad_f32(const void* x, int x_bf16, const float* dz, int N, int H, int W, int Ci, int Co, float* slabs,
              int* nslabs, hipStream_t s) {
  const long R = (long)N * H;
  const int chunks = wgrad_f32_chunks(N, H);
  const int rpc = (int)((R + chunks - 1) / chunks);
  const int nch = (int)((R + rpc - 1) / rpc);
  const long E = 9L * Ci * Co;
  dim3 grid((unsigned)((E + 255) / 256), nch);
  if (x_bf16)
    hipLaunchKernelGGL(k_wgrad_f32<bf16>, grid, dim3(256), 0, s, (const bf16*)x, dz, N, H, W, Ci, Co, rpc, slabs);
  else
    hipLaunchKernelGGL(k_wgrad_f32<float>, grid, dim3(256), 0, s, (const float*)x, dz, N, H, W, Ci, Co, rpc, slabs);
  ASR_LAUNCH_CHECK("k_wgrad_f32");
  if (Co > 1024) return fail(ASR_E_UNSUPPORTED, "db: C > 1024");
  hipLaunchKernelGGL(k_db_f32, dim3(nch), dim3(((Co + 63) / 64) * 64), 0, s, dz, R, W, Co, rpc, E, slabs);
  ASR_LAUNCH_CHECK("k_db_f32");
  *nslabs = nch;
  return ASR_OK;
}

}  // namespace asr
