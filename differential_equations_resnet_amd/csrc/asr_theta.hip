// Parametrisation of the antisymmetric kernel: theta -> W materialisation and
// the dW -> dtheta pull-back.
//
// Reference: layers/tfkeras_layer_Conv2DAntisymmetric3By3.py:104-141 (assembly
// loop, one slice/neg/concat graph per output channel) and :210-293 (diagonal
// block [[a,b,c],[d,gamma,-d],[-c,-b,-a]], off-diagonal -rot180 transpose);
// layers/tfkeras_layer_Conv2DAntisymmetric.py:109-145, :216-270 (general layer).
//
// Instead of ~24(C-1)+1.5C(C-1) graph ops per layer per step, the whole
// assembly is a precomputed element map (asr_param_map, built once on the
// host) and one gather launch for all L layers of a network (asr_theta_to_w).
// The map's transpose gives the exact autodiff of the assembly: every theta
// entry feeds at most two W entries with signs +-1, so dtheta is a two-term
// gather from the reduced dW (k_project).
#include <stdarg.h>
#include <stdio.h>

#include <vector>

#include "asr_common.h"

namespace asr {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int check_ws_device(const void* ws, const char* who) {
  int dev = 0;
  ASR_TRY(hip_check(hipGetDevice(&dev), "hipGetDevice"));
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, ws) != hipSuccess) {
    (void)hipGetLastError();  // (clear the failed query's error)
    return fail(ASR_E_WORKSPACE, "%s: the workspace is not HIP device memory", who);
  }
  if (a.type != hipMemoryTypeDevice || a.device != dev)
    return fail(ASR_E_WORKSPACE,
                "%s: the workspace is not device memory of the current device %d (type %d, device %d): its layout "
                "follows the CU count of the device it was sized on",
                who, dev, (int)a.type, a.device);
  return ASR_OK;
}

int cu_count() {
  static thread_local int dev_cached = -1, cus = 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (dev != dev_cached) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    dev_cached = dev;
    cus = v;
  }
  return cus;
}

// ---------------------------------------------------------------------------
// host: element maps
// ---------------------------------------------------------------------------

// Free positions of the general layer's diagonal block in variable-creation
// order (…Conv2DAntisymmetric.py:231-264), for an odd kernel_size k.
static void general_free_positions(int k, int antisymmetric, std::vector<std::pair<int, int>>& out) {
  for (int i = 0; i < k; ++i)
    for (int j = i; j < k; ++j) {
      if (j > i || (j == i && i <= k / 2 - 1))
        out.push_back({i, j});
      else if (j == i && i == k / 2 && (k % 2) == 1 && !antisymmetric)
        out.push_back({i, j});
    }
}

static bool kernel_size_ok(int kind, int k) {
  return kind == ASR_PARAM_3BY3 ? k == 3 : (k >= 1 && k <= 15 && (k & 1));
}

long theta_count_k(int C, int k, int kind, int antisymmetric) {
  if (C < 1 || !kernel_size_ok(kind, k)) return -1;
  const long kk = (long)k * k;
  if (kind == ASR_PARAM_3BY3) return 4L * C + 9L * C * (C - 1) / 2;
  if (kind == ASR_PARAM_GENERAL) {
    std::vector<std::pair<int, int>> fp;
    general_free_positions(k, antisymmetric, fp);
    return (long)fp.size() * C + kk * C * (C - 1) / 2;
  }
  if (kind == ASR_PARAM_REGULAR) return kk * C * C;
  return -1;
}
long theta_count(int C, int kind, int antisymmetric) { return theta_count_k(C, 3, kind, antisymmetric); }

// The element map of a k x k layer: w_src[e] (e = ((ky*k + kx)*C + i)*C + o,
// HWIO) = (theta index << 1 | negated), -1 for the gamma centre; theta_dst its
// transpose (<= 2 entries per theta).
int param_map_k(int C, int k, int kind, int antisymmetric, int32_t* w_src, int32_t* theta_dst) {
  if (C < 1 || !w_src) return fail(ASR_E_ARG, "asr_param_map: bad arguments");
  if (kind == ASR_PARAM_3BY3 && !antisymmetric)
    return fail(ASR_E_ARG, "asr_param_map: the 3by3 layer is always antisymmetric");
  if (!kernel_size_ok(kind, k))
    return fail(ASR_E_ARG, "asr_param_map: kernel_size %d (3 for the 3by3 layer, odd 1..15 otherwise)", k);
  const long E = (long)k * k * C * C;
  auto idx = [C, k](int ky, int kx, int i, int o) { return ((long)(ky * k + kx) * C + i) * C + o; };
  for (long e = 0; e < E; ++e) w_src[e] = -1;  // gamma unless set below
  if (kind == ASR_PARAM_3BY3) {
    // diagonal: a (0,0) b (0,1) c (0,2) d (1,0); mirrors negated (…3By3.py:261-275)
    const int pos[8][2] = {{0, 0}, {0, 1}, {0, 2}, {1, 0}, {2, 2}, {2, 1}, {2, 0}, {1, 2}};
    const int var[8] = {0, 1, 2, 3, 0, 1, 2, 3};
    const int neg[8] = {0, 0, 0, 0, 1, 1, 1, 1};
    for (int o = 0; o < C; ++o)
      for (int q = 0; q < 8; ++q)
        w_src[idx(pos[q][0], pos[q][1], o, o)] = (int32_t)(((long)(var[q] * C + o) << 1) | neg[q]);
    long base = 4L * C;
    for (int o = 0; o < C - 1; ++o) {
      const int nind = C - o - 1;
      for (int i = o + 1; i < C; ++i) {
        const int m = i - o - 1;
        for (int ky = 0; ky < 3; ++ky)
          for (int kx = 0; kx < 3; ++kx) {
            const long j = base + (long)(ky * 3 + kx) * nind + m;
            w_src[idx(ky, kx, i, o)] = (int32_t)(j << 1);                  // W[:,:,i,o] = indep_o
            w_src[idx(2 - ky, 2 - kx, o, i)] = (int32_t)((j << 1) | 1);    // W[:,:,o,i] = -rot180
          }
      }
      base += 9L * nind;
    }
  } else if (kind == ASR_PARAM_GENERAL) {
    std::vector<std::pair<int, int>> fp;
    general_free_positions(k, antisymmetric, fp);
    long off = 0;
    for (int o = 0; o < C; ++o) {
      for (size_t n = 0; n < fp.size(); ++n) {
        const int i = fp[n].first, j = fp[n].second;
        const long t = off + (long)n;
        w_src[idx(i, j, o, o)] = (int32_t)(t << 1);
        const int mi = k - 1 - i, mj = k - 1 - j;
        if (mi != i || mj != j) w_src[idx(mi, mj, o, o)] = (int32_t)((t << 1) | (antisymmetric ? 1 : 0));
      }
      off += (long)fp.size();
      const int nind = C - o - 1;
      if (nind > 0) {
        for (int i = o + 1; i < C; ++i) {
          const int m = i - o - 1;
          for (int ky = 0; ky < k; ++ky)
            for (int kx = 0; kx < k; ++kx) {
              const long j = off + (long)(ky * k + kx) * nind + m;  // [k,k,nind,1]
              w_src[idx(ky, kx, i, o)] = (int32_t)(j << 1);
              w_src[idx(k - 1 - ky, k - 1 - kx, o, i)] = (int32_t)((j << 1) | 1);  // -J K J (:139)
            }
        }
        off += (long)k * k * nind;
      }
    }
  } else if (kind == ASR_PARAM_REGULAR) {
    for (long e = 0; e < E; ++e) w_src[e] = (int32_t)(e << 1);
  } else {
    return fail(ASR_E_ARG, "asr_param_map: unknown kind %d", kind);
  }
  if (theta_dst) {
    const long nt = theta_count_k(C, k, kind, antisymmetric);
    for (long j = 0; j < 2 * nt; ++j) theta_dst[j] = -1;
    for (long e = 0; e < E; ++e) {
      const int32_t v = w_src[e];
      if (v < 0) continue;
      const long j = v >> 1;
      const int32_t enc = (int32_t)((e << 1) | (v & 1));
      if (theta_dst[2 * j] < 0)
        theta_dst[2 * j] = enc;
      else if (theta_dst[2 * j + 1] < 0)
        theta_dst[2 * j + 1] = enc;
      else
        return fail(ASR_E_ARG, "asr_param_map: theta %ld feeds more than two W entries", j);
    }
  }
  return ASR_OK;
}

int param_map(int C, int kind, int antisymmetric, int32_t* w_src, int32_t* theta_dst) {
  return param_map_k(C, 3, kind, antisymmetric, w_src, theta_dst);
}

int param_is_antisymmetric(int kind, int antisymmetric) {
  if (kind == ASR_PARAM_3BY3) return 1;
  if (kind == ASR_PARAM_GENERAL) return antisymmetric ? 1 : 0;
  if (kind == ASR_PARAM_REGULAR) return 0;
  return fail(ASR_E_ARG, "asr_param_is_antisymmetric: unknown kind %d", kind);
}

// W_bwd[ky,kx,i,o] = -W[k-1-ky,k-1-kx,o,i]: conv(dz, W_bwd) = -A^T dz, so the
// backward's dx = dy - conv(dz, W_bwd) (+ 2*0*dz) is dy + A^T dz for any W.
int param_map_transpose_k(int C, int k, const int32_t* w_src, int32_t* w_bwd) {
  if (C < 1 || k < 1 || !w_src || !w_bwd) return fail(ASR_E_ARG, "asr_param_map_transpose: bad arguments");
  auto idx = [C, k](int ky, int kx, int i, int o) { return ((long)(ky * k + kx) * C + i) * C + o; };
  for (int ky = 0; ky < k; ++ky)
    for (int kx = 0; kx < k; ++kx)
      for (int i = 0; i < C; ++i)
        for (int o = 0; o < C; ++o) {
          const int32_t v = w_src[idx(k - 1 - ky, k - 1 - kx, o, i)];
          if (v < 0) return fail(ASR_E_ARG, "asr_param_map_transpose: map has constant (gamma) entries");
          w_bwd[idx(ky, kx, i, o)] = v ^ 1;
        }
  return ASR_OK;
}
int param_map_transpose(int C, const int32_t* w_src, int32_t* w_bwd) { return param_map_transpose_k(C, 3, w_src, w_bwd); }

// ---------------------------------------------------------------------------
// device: materialisation
// ---------------------------------------------------------------------------

__device__ __forceinline__ float w_value(const float* theta, const int32_t* w_src, long e, float gamma) {
  const int32_t v = w_src[e];
  if (v < 0) return gamma;
  const float t = theta[v >> 1];
  return (v & 1) ? -t : t;
}

// plain HWIO float (E = k*k*C*C elements): one thread per element, blockIdx.y = layer
__global__ void k_theta_to_w_hwio(const float* __restrict__ theta, long theta_stride, long E,
                                  const int32_t* __restrict__ w_src, float gamma, float* __restrict__ w,
                                  long w_stride) {
  const int l = blockIdx.y;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < E; e += (long)gridDim.x * blockDim.x)
    w[l * w_stride + e] = w_value(theta + l * theta_stride, w_src, e, gamma);
}

// MFMA fragment-packed bf16 (see asr_conv_mfma.hip, "W pack"):
//   pack[((ot*KS + ks)*64 + lane)*8 + j] = W^T[o = 16*ot + (lane&15)][kappa = 32*ks + 8*(lane>>4) + j]
//   with kappa = tap*C + i (tap = ky*3+kx), zero for kappa >= 9C.
// One 64-lane wave per (ot, ks) fragment: each lane builds its 8 elements and
// writes 16 contiguous bytes.
// w_lo (nullable): the residual bf16(W - float(bf16(W))) in the same packing
// (the hi/lo weight split of k_fwd16_fused).
__global__ void k_theta_to_w_pack(const float* __restrict__ theta, long theta_stride, int C,
                                  const int32_t* __restrict__ w_src, float gamma, bf16* __restrict__ w,
                                  long w_stride, bf16* __restrict__ w_lo) {
  const int KS = (9 * C + 31) / 32;
  const int OT = C / 16;
  const int l = blockIdx.y;
  const int frag = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  if (frag >= OT * KS) return;
  const int lane = threadIdx.x & 63;
  const int ot = frag / KS, ks = frag % KS;
  const int o = 16 * ot + (lane & 15);
  const float* th = theta + l * theta_stride;
  bf16x8 v, vl;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int kappa = 32 * ks + 8 * (lane >> 4) + j;
    float x = 0.f;
    if (kappa < 9 * C) {
      const int tap = kappa / C, i = kappa % C;
      x = w_value(th, w_src, ((long)tap * C + i) * C + o, gamma);
    }
    v[j] = (bf16)x;
    vl[j] = (bf16)(x - (float)v[j]);
  }
  *(bf16x8*)(w + l * w_stride + ((long)frag * 64 + lane) * 8) = v;
  if (w_lo) *(bf16x8*)(w_lo + l * w_stride + ((long)frag * 64 + lane) * 8) = vl;
}

// ---------------------------------------------------------------------------
// device: split-K reduction of fp32 slabs and the theta projection
// ---------------------------------------------------------------------------

// out[g][e] = sum_{p in [g*per, min((g+1)*per, P))} in[p][e]   (deterministic)
__global__ void k_reduce_slabs(const float* __restrict__ in, long E, int P, int per, float* __restrict__ out) {
  const long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const int g = blockIdx.y;
  if (e >= E) return;
  const int p0 = g * per, p1 = min(P, p0 + per);
  float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
  int p = p0;
  for (; p + 3 < p1; p += 4) {
    acc0 += in[(long)p * E + e];
    acc1 += in[(long)(p + 1) * E + e];
    acc2 += in[(long)(p + 2) * E + e];
    acc3 += in[(long)(p + 3) * E + e];
  }
  for (; p < p1; ++p) acc0 += in[(long)p * E + e];
  out[(long)g * E + e] = (acc0 + acc1) + (acc2 + acc3);
}

// dtheta[j] = sum over the (<=2) W entries theta j feeds of sign * dW[e],
// from the fully reduced slab row [dW (E floats) | db (Cb floats)].  Also an
// optional dW copy and db.
__global__ void k_project(const float* __restrict__ red_groups, int G, long E, const int32_t* __restrict__ theta_dst,
                          long n_theta, float* __restrict__ dtheta, float* __restrict__ dw_out, int Cb,
                          float* __restrict__ dbias) {
  const long t = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const long ES = E + Cb;
  auto red_at = [&](long e) {  // sum of the G group partials (fixed order: deterministic)
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    int g = 0;
    for (; g + 3 < G; g += 4) {  // four independent loads in flight
#pragma unroll
      for (int q = 0; q < 4; ++q) a[q] += red_groups[(long)(g + q) * ES + e];
    }
    for (; g < G; ++g) a[0] += red_groups[(long)g * ES + e];
    return (a[0] + a[1]) + (a[2] + a[3]);
  };
  if (dtheta && t < n_theta) {
    float acc = 0.f;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int32_t v = theta_dst[2 * t + q];
      if (v >= 0) {
        const float d = red_at(v >> 1);
        acc += (v & 1) ? -d : d;
      }
    }
    dtheta[t] = acc;
  }
  if (dw_out && t < E) dw_out[t] = red_at(t);
  if (dbias && t < Cb) dbias[t] = red_at(E + t);
}

int theta_dst_pair_host(const int32_t* in, long n_theta, int C, int32_t* out);  // (below)

}  // namespace asr

using namespace asr;

extern "C" {

const char* asr_last_error(void) { return g_err; }
int asr_abi_version(void) { return 8; }

int asr_device_cu_count(void) { return cu_count(); }

long asr_theta_count(int C, int kind, int antisymmetric) { return theta_count(C, kind, antisymmetric); }
long asr_theta_count_k(int C, int kernel_size, int kind, int antisymmetric) {
  return theta_count_k(C, kernel_size, kind, antisymmetric);
}
int asr_param_map_k(int C, int kernel_size, int kind, int antisymmetric, int32_t* w_src, int32_t* theta_dst) {
  return param_map_k(C, kernel_size, kind, antisymmetric, w_src, theta_dst);
}
int asr_param_map_transpose_k(int C, int kernel_size, const int32_t* w_src, int32_t* w_src_bwd) {
  return param_map_transpose_k(C, kernel_size, w_src, w_src_bwd);
}

int asr_param_map(int C, int kind, int antisymmetric, int32_t* w_src, int32_t* theta_dst) {
  return param_map(C, kind, antisymmetric, w_src, theta_dst);
}

int asr_param_is_antisymmetric(int kind, int antisymmetric) { return param_is_antisymmetric(kind, antisymmetric); }

int asr_param_map_transpose(int C, const int32_t* w_src, int32_t* w_src_bwd) {
  return param_map_transpose(C, w_src, w_src_bwd);
}

int asr_param_map_pair(int C, const int32_t* theta_dst, long n_theta, int32_t* theta_dst_pair) {
  if (C != 64 || !theta_dst || !theta_dst_pair || n_theta < 0)
    return fail(ASR_E_ARG, "asr_param_map_pair: C=64 and non-null maps required");
  return theta_dst_pair_host(theta_dst, n_theta, C, theta_dst_pair);
}

long asr_wpack_elems(int C) {
  if (C % 16 != 0) return -1;
  return (long)(C / 16) * ((9 * C + 31) / 32) * 64 * 8;
}

int asr_theta_to_w_k(const float* theta, long theta_stride, int L, int C, int kernel_size, const int32_t* w_src,
                     float gamma, float* w_out, long w_stride, asr_stream_t stream) {
  if (!theta || !w_src || !w_out || L < 1 || C < 1 || L > 65535 || kernel_size < 1)
    return fail(ASR_E_ARG, "asr_theta_to_w_k: bad arguments");
  const long E = (long)kernel_size * kernel_size * C * C;
  if (w_stride < E) return fail(ASR_E_ARG, "asr_theta_to_w_k: w_stride too small");
  dim3 grid((unsigned)std::min<long>((E + 255) / 256, 1024), L);
  hipLaunchKernelGGL(k_theta_to_w_hwio, grid, dim3(256), 0, (hipStream_t)stream, theta, theta_stride, E, w_src, gamma,
                     w_out, w_stride);
  ASR_LAUNCH_CHECK("k_theta_to_w_hwio");
  return ASR_OK;
}

int asr_theta_to_w(const float* theta, long theta_stride, int L, int C, const int32_t* w_src, float gamma,
                   void* w_out, long w_stride, int dtype, asr_stream_t stream) {
  if (!theta || !w_src || !w_out || L < 1 || C < 1 || L > 65535)
    return fail(ASR_E_ARG, "asr_theta_to_w: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  if (dtype == ASR_F32) {
    const long E = 9L * C * C;
    if (w_stride < E) return fail(ASR_E_ARG, "asr_theta_to_w: w_stride too small");
    dim3 grid((unsigned)std::min<long>((E + 255) / 256, 1024), L);
    hipLaunchKernelGGL(k_theta_to_w_hwio, grid, dim3(256), 0, s, theta, theta_stride, E, w_src, gamma,
                       (float*)w_out, w_stride);
    ASR_LAUNCH_CHECK("k_theta_to_w_hwio");
  } else if (dtype == ASR_BF16) {
    if (C % 16 != 0) return fail(ASR_E_UNSUPPORTED, "asr_theta_to_w: bf16 pack needs C %% 16 == 0 (C=%d)", C);
    if (w_stride < asr_wpack_elems(C)) return fail(ASR_E_ARG, "asr_theta_to_w: w_stride too small");
    const int frags = (C / 16) * ((9 * C + 31) / 32);
    dim3 grid((frags + 3) / 4, L);
    hipLaunchKernelGGL(k_theta_to_w_pack, grid, dim3(256), 0, s, theta, theta_stride, C, w_src, gamma,
                       (bf16*)w_out, w_stride, (bf16*)nullptr);
    ASR_LAUNCH_CHECK("k_theta_to_w_pack");
  } else {
    return fail(ASR_E_ARG, "asr_theta_to_w: bad dtype %d", dtype);
  }
  return ASR_OK;
}

}  // extern "C"

namespace asr {

// asr_theta_to_w's bf16 pack plus the residual pack w_lo = bf16(W - bf16(W))
// (the hi/lo operands of the fused C=16 forward, k_fwd16_fused<.., LO>)
int theta_to_w_pack_hilo(const float* theta, long theta_stride, int L, int C, const int32_t* w_src, float gamma,
                         void* w_hi, void* w_lo, long w_stride, hipStream_t s) {
  if (!theta || !w_src || !w_hi || !w_lo || L < 1 || L > 65535 || C % 16 != 0 || w_stride < asr_wpack_elems(C))
    return fail(ASR_E_ARG, "theta_to_w_pack_hilo: bad arguments");
  const int frags = (C / 16) * ((9 * C + 31) / 32);
  hipLaunchKernelGGL(k_theta_to_w_pack, dim3((frags + 3) / 4, L), dim3(256), 0, s, theta, theta_stride, C, w_src,
                     gamma, (bf16*)w_hi, w_stride, (bf16*)w_lo);
  ASR_LAUNCH_CHECK("k_theta_to_w_pack");
  return ASR_OK;
}

// Reduce P slab rows of ES = E + Cb floats ([dW partial | db partial], written
// by the wgrad kernels) deterministically in two passes (P -> ceil(P/32) -> 1),
// then project dW onto theta (if theta_dst) and/or copy dW / db out.
// ws must hold reduce_ws_bytes(P, E + Cb) bytes.
int reduce_and_project(const float* slabs, int P, long E, int Cb, const int32_t* theta_dst, long n_theta,
                       float* dtheta, float* dbias, float* dw_out, float* ws, hipStream_t s) {
  const long ES = E + Cb;
  const int per = 32;
  const int G = (P + per - 1) / per;
  float* grp = ws;
  float* fin = ws + (long)G * ES;
  dim3 g1((unsigned)((ES + 255) / 256), G);
  hipLaunchKernelGGL(k_reduce_slabs, g1, dim3(256), 0, s, slabs, ES, P, per, grp);
  ASR_LAUNCH_CHECK("k_reduce_slabs");
  (void)fin;
  const long n = std::max(std::max(dtheta ? n_theta : 0L, dw_out ? E : 0L), (long)Cb);
  hipLaunchKernelGGL(k_project, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, grp, G, E, theta_dst,
                     dtheta ? n_theta : 0L, dtheta, dw_out, Cb, dbias);
  ASR_LAUNCH_CHECK("k_project");
  return ASR_OK;
}

size_t reduce_ws_bytes(int P, long ES) { return (size_t)((P + 31) / 32 + 1) * ES * sizeof(float); }

int reduce_groups(int P) { return (P + 31) / 32; }

// Pass 1 for L layers in one launch: layer z's P slab rows at slabs + z*slab_stride -> its
// reduce_groups(P) group rows at grp + z*grp_stride (the fp32 network's per-block slabs)
__global__ void k_reduce_slabs_layers(const float* __restrict__ in, long slab_stride, long E, int P, int per,
                                      float* __restrict__ out, long out_stride) {
  const long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const int g = blockIdx.y;
  if (e >= E) return;
  const float* src = in + blockIdx.z * slab_stride;
  const int p0 = g * per, p1 = min(P, p0 + per);
  float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
  int p = p0;
  for (; p + 3 < p1; p += 4) {
    acc0 += src[(long)p * E + e];
    acc1 += src[(long)(p + 1) * E + e];
    acc2 += src[(long)(p + 2) * E + e];
    acc3 += src[(long)(p + 3) * E + e];
  }
  for (; p < p1; ++p) acc0 += src[(long)p * E + e];
  out[blockIdx.z * out_stride + (long)g * E + e] = (acc0 + acc1) + (acc2 + acc3);
}

int reduce_slab_layers(const float* slabs, long slab_stride, int P, long ES, float* grp, long grp_stride, int L,
                       hipStream_t s) {
  if (L < 1 || P < 1) return ASR_OK;
  dim3 g1((unsigned)((ES + 255) / 256), reduce_groups(P), L);
  hipLaunchKernelGGL(k_reduce_slabs_layers, g1, dim3(256), 0, s, slabs, slab_stride, ES, P, 32, grp, grp_stride);
  ASR_LAUNCH_CHECK("k_reduce_slabs_layers");
  return ASR_OK;
}

// Pass 1 only: P slab rows of ES floats -> reduce_groups(P) group rows at grp.
int reduce_slabs_to_groups(const float* slabs, int P, long ES, float* grp, hipStream_t s) {
  const int G = reduce_groups(P);
  dim3 g1((unsigned)((ES + 255) / 256), G);
  hipLaunchKernelGGL(k_reduce_slabs, g1, dim3(256), 0, s, slabs, ES, P, 32, grp);
  ASR_LAUNCH_CHECK("k_reduce_slabs");
  return ASR_OK;
}

// Pass 2 + projection for L layers in one launch: layer l's G group rows of
// [dW (E) | db (Cb)] at grp + l*grp_stride -> dtheta at out + l*out_stride,
// db right after it (the network's [theta | bias] block layout).
__global__ void k_project_layers(const float* __restrict__ grp, long grp_stride, int G, long E, int Cb,
                                 const int32_t* __restrict__ theta_dst, long n_theta, float* __restrict__ out,
                                 long out_stride) {
  const int l = blockIdx.y;
  const float* rg = grp + (long)l * grp_stride;
  const long ES = E + Cb;
  const long t = blockIdx.x * (long)blockDim.x + threadIdx.x;
  auto red_at = [&](long e) {
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    int g = 0;
    for (; g + 3 < G; g += 4) {
#pragma unroll
      for (int q = 0; q < 4; ++q) a[q] += rg[(long)(g + q) * ES + e];
    }
    for (; g < G; ++g) a[0] += rg[(long)g * ES + e];
    return (a[0] + a[1]) + (a[2] + a[3]);
  };
  float* o = out + (long)l * out_stride;
  if (t < n_theta) {
    const int32_t v0 = theta_dst[2 * t], v1 = theta_dst[2 * t + 1];
    float acc = 0.f;
    if (v0 >= 0) acc += (v0 & 1) ? -red_at(v0 >> 1) : red_at(v0 >> 1);
    if (v1 >= 0) acc += (v1 & 1) ? -red_at(v1 >> 1) : red_at(v1 >> 1);
    o[t] = acc;
  } else if (t < n_theta + Cb) {
    o[t] = red_at(E + (t - n_theta));
  }
}

// rows [l][0] = sum_g grp[l][g] (coalesced, fixed order), in place
__global__ void k_sum_groups(float* __restrict__ grp, long grp_stride, int G, long ES) {
  const long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (e >= ES) return;
  float* rg = grp + (long)blockIdx.y * grp_stride;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  int g = 0;
  for (; g + 3 < G; g += 4) {
#pragma unroll
    for (int q = 0; q < 4; ++q) a[q] += rg[(long)(g + q) * ES + e];
  }
  for (; g < G; ++g) a[0] += rg[(long)g * ES + e];
  rg[e] = (a[0] + a[1]) + (a[2] + a[3]);
}

// theta_dst entries (e<<1)|neg with e = m*C + o (dW row-major) -> the same
// entries into the tile-major dW of k_bwd3_stack's slabs:
// ((m/16 * C/16 + o/16) * 64 + 16*((m%16)/4) + o%16) * 4 + m%4
__global__ void k_theta_dst_tile(const int32_t* __restrict__ in, long n, int C, int32_t* __restrict__ out) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t v = in[i];
  if (v < 0) {
    out[i] = v;
    return;
  }
  const long e = v >> 1, m = e / C, o = e % C;
  const long et = (((m / 16) * (C / 16) + o / 16) * 64 + 16 * ((m % 16) / 4) + o % 16) * 4 + m % 4;
  out[i] = (int32_t)((et << 1) | (v & 1));
}

// theta_dst (pairs of (e << 1 | neg) entries per theta, asr_param_map) of an
// antisymmetric parametrisation -> the same pull-back from the pair-local
// slabs (pair_encode of the first entry: the second is its mirror)
__global__ void k_theta_dst_pair(const int32_t* __restrict__ in, long n_theta, int C, int32_t* __restrict__ out) {
  const long j = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (j >= n_theta) return;
  int32_t o[2] = {-1, -1};
  const int32_t v = in[2 * j];
  if (v >= 0) pair_encode(v >> 1, v & 1, C, o);
  out[2 * j] = o[0];
  out[2 * j + 1] = o[1];
}

int theta_dst_pair(const int32_t* in, long n_theta, int C, int32_t* out, hipStream_t s) {
  if (C != 64) return fail(ASR_E_UNSUPPORTED, "pair-local slabs: C=64 only");
  hipLaunchKernelGGL(k_theta_dst_pair, dim3((unsigned)((n_theta + 255) / 256)), dim3(256), 0, s, in, n_theta, C, out);
  ASR_LAUNCH_CHECK("k_theta_dst_pair");
  return ASR_OK;
}

// host: the same from a host theta_dst; ASR_E_ARG when some theta is not an
// antisymmetric pair (e, mirror(e)) with opposite signs (the pair-local path
// does not apply)
int theta_dst_pair_host(const int32_t* in, long n_theta, int C, int32_t* out) {
  for (long j = 0; j < n_theta; ++j) {
    const int32_t v0 = in[2 * j], v1 = in[2 * j + 1];
    if (v0 < 0 || v1 < 0) return fail(ASR_E_ARG, "theta %ld: not an antisymmetric pair", j);
    const long e0 = v0 >> 1, e1 = v1 >> 1;
    const int t = (int)(e0 / ((long)C * C)), i = (int)((e0 / C) % C), o = (int)(e0 % C);
    const long mirror = ((long)(8 - t) * C + o) * C + i;
    if (e1 != mirror || ((v0 ^ v1) & 1) == 0) return fail(ASR_E_ARG, "theta %ld: not an antisymmetric pair", j);
    int32_t o2[2] = {-1, -1};
    if (pair_encode(e0, v0 & 1, C, o2) == 0) return fail(ASR_E_ARG, "theta %ld: no pair-local slab entry", j);
    out[2 * j] = o2[0];
    out[2 * j + 1] = o2[1];
  }
  return ASR_OK;
}

int theta_dst_tile_major(const int32_t* in, long n, int C, int32_t* out, hipStream_t s) {
  hipLaunchKernelGGL(k_theta_dst_tile, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in, n, C, out);
  ASR_LAUNCH_CHECK("k_theta_dst_tile");
  return ASR_OK;
}

int project_layers(float* grp, long grp_stride, int G, long E, int Cb, const int32_t* theta_dst, long n_theta,
                   int L, float* out, long out_stride, hipStream_t s) {
  const long n = n_theta + Cb;
  if (G > 1) {  // pass 2 coalesced, then the projection gathers from one row per layer
    hipLaunchKernelGGL(k_sum_groups, dim3((unsigned)((E + Cb + 255) / 256), L), dim3(256), 0, s, grp, grp_stride, G,
                       E + Cb);
    ASR_LAUNCH_CHECK("k_sum_groups");
  }
  hipLaunchKernelGGL(k_project_layers, dim3((unsigned)((n + 255) / 256), L), dim3(256), 0, s, grp, grp_stride, 1, E,
                     Cb, theta_dst, n_theta, out, out_stride);
  ASR_LAUNCH_CHECK("k_project_layers");
  return ASR_OK;
}

}  // namespace asr
