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

#include <algorithm>
#include <type_traits>
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
// writes 16 contiguous bytes.  Round to nearest (the pack of C > 64, and of
// ASR_VARIANT_W_BF16).
__global__ void k_theta_to_w_pack(const float* __restrict__ theta, long theta_stride, int C,
                                  const int32_t* __restrict__ w_src, float gamma, bf16* __restrict__ w,
                                  long w_stride) {
  const int KS = (9 * C + 31) / 32;
  const int OT = C / 16;
  const int l = blockIdx.y;
  const int frag = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  if (frag >= OT * KS) return;
  const int lane = threadIdx.x & 63;
  const int ot = frag / KS, ks = frag % KS;
  const int o = 16 * ot + (lane & 15);
  const float* th = theta + l * theta_stride;
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int kappa = 32 * ks + 8 * (lane >> 4) + j;
    float x = 0.f;
    if (kappa < 9 * C) {
      const int tap = kappa / C, i = kappa % C;
      x = w_value(th, w_src, ((long)tap * C + i) * C + o, gamma);
    }
    v[j] = (bf16)x;
  }
  *(bf16x8*)(w + l * w_stride + ((long)frag * 64 + lane) * 8) = v;
}

// Balanced rounding of the bf16 pack (C in {16, 32, 64}).
// Rounding W to nearest perturbs output channel o by the fixed sum of its
// row's rounding errors, which every pixel of every image and every layer of a
// deep stack sees the same way; over C3's 108 blocks that coherent error is
// the bf16 path's largest deviation from the fp32 reference (group rel-L2
// 2.6e-2 from W alone, tools/bf16_depth_emulate.py).  Where the map pairs
// every off-diagonal entry with its antisymmetric partner (W[t][i][o] =
// -W[8-t][o][i], one theta: the 3by3 and general kinds), each pair instead
// takes the bf16 neighbour (below or above) that keeps the two channels'
// error sums e_o, e_i smallest -- cost (e_o + d)^2 + (e_i - d)^2, i.e. the
// upper neighbour iff D + (d_lo + d_hi) < 0 with D = e_o - e_i, else the lower
// one (an entry that is a bf16 value already stays).  The pack stays exactly
// antisymmetric (both entries of a pair from one q) and is still a bf16 W: the
// conv kernels are unchanged.  The pairs go in C-1 rounds of C/2 disjoint
// channel pairs (the round-robin circle schedule, one lane per pair); within a
// pair, taps 0..8 in order with D += 2d per tap, then e_o += S, e_i -= S for
// the pair's S = sum d (all fp32); each channel's sum starts from its
// diagonal entries rounded to nearest (taps 0..8; the centre gamma, and the
// mirrored diagonal pairs of the non-antisymmetric general kind);
// tests/helpers.py w_bf16_balanced restates it bit-exactly.
__device__ __forceinline__ unsigned wpack_pos(int KS, int o, int kappa) {
  const int r = kappa & 31;
  return (unsigned)((((o >> 4) * KS + (kappa >> 5)) * 64 + (o & 15) + 16 * (r >> 3)) * 8 + (r & 7));
}

constexpr int kBalThreads = 1024;

// the round-robin pair schedule: round r, slot p -> channels o < i
template <int C>
__device__ __forceinline__ void bal_pair(int r, int p, int& o, int& i) {
  const int a = p == 0 ? C - 1 : (r + p) % (C - 1), b = p == 0 ? r : (r - p + (C - 1)) % (C - 1);
  o = min(a, b);
  i = max(a, b);
}

template <int C>
__device__ __forceinline__ int bal_slot(int o, int i) {  // (r * C/2 + p) of the pair o < i
  if (i == C - 1) return o * (C / 2);
  const int r = ((o + i) * (C / 2)) % (C - 1);  // (2 (C/2) = 1 mod C-1)
  return r * (C / 2) + min((o - r + (C - 1)) % (C - 1), (i - r + (C - 1)) % (C - 1));
}

// The kernel: one workgroup per layer.  (1) In schedule order (round r, pair
// slot p, tap t), every pair's lower entry W[t][i][o] (i > o) into LDS, with
// the pairing check of the map; the diagonal rounded to nearest straight into
// the pack (a map without the pairing: every entry to nearest, and done).  (2)
// Barrier-separated steps of R rounds: wave 0 runs the error chain of the
// previous step's rounds (per tap: one 16-B read of the precomputed
// candidates, the decision, the error sums; R rounds without a barrier, LDS
// in program order within the wave) while the waves on the other three SIMDs
// precompute the next step's candidates {d_lo + d_hi, d_lo, d_hi} and
// write the decided pairs (q, -q) of the step before into the pack.
template <int C>
__device__ __forceinline__ void pack_bal_layer(const float* __restrict__ theta, long theta_stride,
                                               const int32_t* __restrict__ w_src, float gamma, bf16* __restrict__ w,
                                               long w_stride, const int32_t* __restrict__ theta_dst, long n_theta,
                                               int l, unsigned char* lds) {
  constexpr int KS = (9 * C + 31) / 32, LC = C == 16 ? 4 : C == 32 ? 5 : 6, NP = C / 2, NR = C - 1;
  constexpr int NQ = NR * NP * 9, NIT = (NQ + kBalThreads - 1) / kBalThreads, NB = NIT < 9 ? NIT : 9;
  constexpr int R = C == 64 ? 4 : 2, NS = (NR + R - 1) / R, SQ = R * NP * 9;  // rounds / records per step
  static_assert(C == 16 || C == 32 || C == 64, "balanced pack: C in {16, 32, 64}");
  f32x4* rec = (f32x4*)lds;          // [3][SQ] {d_lo + d_hi, d_lo, d_hi, -}
  float* dec = (float*)(rec + 3 * SQ);  // [3][SQ] the chosen d
  float* xr = dec + 3 * SQ;           // [NQ] the pairs' lower entries, schedule order ((r * NP + p) * 9 + t)
  float* err = xr + NQ;               // [C] per output channel: its rounding errors' sum
  const int tid = threadIdx.x;
  const float* th = theta + l * theta_stride;
  bf16* wl = w + l * w_stride;
  auto pos = [](int o, int kappa) { return wpack_pos(KS, o, kappa); };
  // 1. the pairs' lower entries, branch-free in batches of NB (a conditional load waits for the one before)
  bool paired = true;
  if (theta_dst) {  // a map known to pair (asr_param_map 3by3 / general): theta and its two entries, coalesced
    for (long j0 = tid; j0 < n_theta; j0 += 4L * kBalThreads) {
      float x[4];
      int32_t a[4], b2[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const long j = min(j0 + (long)k * kBalThreads, n_theta - 1);
        x[k] = th[j];
        a[k] = theta_dst[2 * j];
        b2[k] = theta_dst[2 * j + 1];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (j0 + (long)k * kBalThreads >= n_theta) break;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int32_t v = h ? b2[k] : a[k];
          if (v < 0) continue;
          const int e = v >> 1, t = e >> (2 * LC), i = (e >> LC) & (C - 1), o = e & (C - 1);
          if (i > o) xr[bal_slot<C>(o, i) * 9 + t] = (v & 1) ? -x[k] : x[k];
        }
      }
    }
  } else {
#pragma unroll
  for (int k0 = 0; k0 < NIT; k0 += NB) {
    int32_t v[NB], v2[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int q = min(tid + (k0 + k) * kBalThreads, NQ - 1), t = q % 9, rp = q / 9;
      int o, i;
      bal_pair<C>(rp / NP, rp % NP, o, i);
      v[k] = w_src[(t * C + i) * C + o];
      v2[k] = w_src[((8 - t) * C + o) * C + i];  // its antisymmetric partner
    }
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const float x = th[max(v[k], 0) >> 1];
      const int q = tid + (k0 + k) * kBalThreads;
      if (k0 + k < NIT && q < NQ) {
        paired = paired && v[k] >= 0 && v2[k] == (v[k] ^ 1);
        xr[q] = (v[k] & 1) ? -x : x;
      }
    }
  }
  }
  for (int e = tid; e < 9 * C; e += kBalThreads) {  // the diagonal: to nearest, into the pack
    const int t = e / C, o = e % C;
    const int32_t v = w_src[(t * C + o) * C + o];
    wl[pos(o, t * C + o)] = (bf16)(v < 0 ? gamma : ((v & 1) ? -th[v >> 1] : th[v >> 1]));
  }
  for (int e = tid; e < C * (32 * KS - 9 * C); e += kBalThreads)  // the pack's zero rows (kappa >= 9C)
    wl[pos(e % C, 9 * C + e / C)] = (bf16)0.f;
  paired = __syncthreads_and(paired);  // (also: xr complete)
  if (!paired) {  // every entry to nearest
    for (int e = tid; e < 9 * C * C; e += kBalThreads) {
      const int tap = e >> (2 * LC), i = (e >> LC) & (C - 1), o = e & (C - 1);
      const int32_t v = w_src[e];
      wl[pos(o, tap * C + i)] = (bf16)(v < 0 ? gamma : ((v & 1) ? -th[v >> 1] : th[v >> 1]));
    }
    return;
  }
  if (tid < C) {  // the sums start from the diagonal entries' (nearest) rounding errors, taps 0..8
    float e = 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int32_t v = w_src[(t * C + tid) * C + tid];
      const float x = v < 0 ? gamma : ((v & 1) ? -th[v >> 1] : th[v >> 1]);
      e = __fadd_rn(e, __fsub_rn((float)(bf16)x, x));
    }
    err[tid] = e;
  }
  __syncthreads();
  // 2. the pipelined steps: step s produces rounds [sR, sR+R), decides [(s-1)R, sR), writes [(s-2)R, (s-1)R)
  if (tid < 64) __builtin_amdgcn_s_setprio(3);  // the chain wave first at its SIMD's issue
  for (int s = 0; s <= NS + 1; ++s) {
    if (tid < 64) {
      if (s >= 1 && s <= NS && tid < NP) {
        const f32x4* rs = rec + ((s - 1) % 3) * SQ;
        float* ds = dec + ((s - 1) % 3) * SQ;
#pragma unroll
        for (int rr = 0; rr < R; ++rr) {
          const int r = (s - 1) * R + rr;
          if (r >= NR) break;
          int o, i;
          bal_pair<C>(r, tid, o, i);
          const f32x4* rc = rs + (rr * NP + tid) * 9;
          float* dc = ds + (rr * NP + tid) * 9;
          // the round's candidates first: a read after a store to the same LDS array waits for the
          // store's turn, so reads interleaved with the decisions' stores cost an LDS latency per tap
          f32x4 c[9];
#pragma unroll
          for (int t = 0; t < 9; ++t) c[t] = rc[t];
          const float eo = err[o], ei = err[i];
          // the chain carries D = e_o - e_i only (4 dependent operations per tap); the pair's total
          // S = sum d moves the two sums at the end
          float D = __fsub_rn(eo, ei), S = 0.f, dv[9];
#pragma unroll
          for (int t = 0; t < 9; ++t) {
            // cost (e_o + d)^2 + (e_i - d)^2: the upper neighbour iff D + (d_lo + d_hi) < 0
            dv[t] = __fadd_rn(D, c[t].x) < 0.f ? c[t].z : c[t].y;
            D = __fmaf_rn(2.f, dv[t], D);  // (2d exact: one rounding)
            S = __fadd_rn(S, dv[t]);
          }
          err[o] = __fadd_rn(eo, S);
          err[i] = __fsub_rn(ei, S);
#pragma unroll
          for (int t = 0; t < 9; ++t) dc[t] = dv[t];
          __builtin_amdgcn_wave_barrier();
        }
      }
    } else if ((tid >> 6) & 3) {  // the producers: the 12 waves off the chain wave's SIMD (768 lanes)
      const int wv = tid >> 6, j0 = ((wv >> 2) * 3 + (wv & 3) - 1) * 64 + (tid & 63);
      for (int j = j0; j < SQ; j += 768) {
        const int q0 = s * SQ + j;  // candidates of step s
        if (s < NS && q0 < NQ) {
          const float x = xr[q0];
          const unsigned bx = __float_as_uint(x);
          const float tz = __uint_as_float(bx & 0xFFFF0000u);            // toward zero
          const float aw = __uint_as_float((bx & 0xFFFF0000u) + 0x10000u);  // away from zero
          const bool exact = (bx & 0xFFFFu) == 0u;  // (a bf16 value already: d = 0 either way)
          const float dtz = __fsub_rn(tz, x), daw = __fsub_rn(aw, x);
          const float d_lo = exact ? 0.f : (x > 0.f ? dtz : daw), d_hi = exact ? 0.f : (x > 0.f ? daw : dtz);
          rec[(s % 3) * SQ + j] = f32x4{exact ? 0.f : __fadd_rn(dtz, daw), d_lo, d_hi, 0.f};
        }
        const int q2 = (s - 2) * SQ + j;  // step s-2 decided: q = x + d (exact: both neighbours are x + d)
        if (s >= 2 && q2 < NQ) {
          const int t = q2 % 9, rp = q2 / 9;
          int o, i;
          bal_pair<C>(rp / NP, rp % NP, o, i);
          const float qv = __fadd_rn(xr[q2], dec[((s - 2) % 3) * SQ + j]);
          wl[pos(o, t * C + i)] = (bf16)qv;
          wl[pos(i, (8 - t) * C + o)] = (bf16)(-qv);
        }
      }
    }
    // LDS-only barrier: __syncthreads would also wait for the pack's global stores every step
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
}

struct PackJobs {
  PackJob j[kMaxPackJobs];
  int n;
};

// one workgroup per layer of every job (block b: job k, layer b - the layers of the jobs before)
__global__ __launch_bounds__(kBalThreads) void k_theta_to_w_pack_bal(PackJobs jobs) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  int b = blockIdx.x, k = 0;
  while (k + 1 < jobs.n && b >= jobs.j[k].L) b -= jobs.j[k++].L;
  const PackJob& J = jobs.j[k];
  const auto args = [&](auto cc) {
    constexpr int C = decltype(cc)::value;
    pack_bal_layer<C>(J.theta, J.theta_stride, J.w_src, J.gamma, (bf16*)J.w, J.w_stride, J.theta_dst, J.n_theta, b,
                      lds);
  };
  if (J.C == 16) args(std::integral_constant<int, 16>{});
  else if (J.C == 32) args(std::integral_constant<int, 32>{});
  else args(std::integral_constant<int, 64>{});
}

static size_t pack_bal_lds(int C) {  // 3 x (candidates + decisions) of a step's R rounds, the pairs' lower entries, the sums
  const int R = C == 64 ? 4 : 2;
  return (size_t)(3 * R * (C / 2) * 9 * 5 + (C - 1) * (C / 2) * 9 + C) * 4;
}

int theta_to_w_bf16_jobs(const PackJob* jobs, int njobs, hipStream_t s) {
  if (njobs < 1 || njobs > kMaxPackJobs) return fail(ASR_E_ARG, "theta_to_w_bf16_jobs: %d jobs", njobs);
  PackJobs pj{};
  size_t lds = 0;
  long blocks = 0;
  for (int k = 0; k < njobs; ++k) {
    const PackJob& J = jobs[k];
    if (!J.theta || !J.w_src || !J.w || J.L < 1 || (J.C != 16 && J.C != 32 && J.C != 64) ||
        J.w_stride < asr_wpack_elems(J.C))
      return fail(ASR_E_ARG, "theta_to_w_bf16_jobs: bad job %d", k);
    pj.j[k] = J;
    lds = std::max(lds, pack_bal_lds(J.C));
    blocks += J.L;
  }
  pj.n = njobs;
  if (blocks > 65535) return fail(ASR_E_ARG, "theta_to_w_bf16_jobs: %ld layers", blocks);
  hipLaunchKernelGGL(k_theta_to_w_pack_bal, dim3((unsigned)blocks), dim3(kBalThreads), lds, s, pj);
  ASR_LAUNCH_CHECK("k_theta_to_w_pack_bal");
  return ASR_OK;
}

// ---------------------------------------------------------------------------
// device: split-K reduction of fp32 slabs and the theta projection
// ---------------------------------------------------------------------------

// The sum of rows [p0, p1) of a slab column (stride E): four accumulators taking rows
// p0 + 4k + j in turn, the remainder into the first, (a0 + a1) + (a2 + a3): a fixed order
// (deterministic).  A full group of 32 rows issues all its loads before the first add
// (a rolled loop kept four in flight: latency-bound at C3's 27648 slab rows).
__device__ __forceinline__ float sum_slab_rows(const float* __restrict__ src, long E, long e, int p0, int p1) {
  float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
  if (p1 - p0 == 32) {
    float v[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) v[k] = src[(long)(p0 + k) * E + e];
#pragma unroll
    for (int k = 0; k < 32; k += 4) {
      acc0 += v[k];
      acc1 += v[k + 1];
      acc2 += v[k + 2];
      acc3 += v[k + 3];
    }
    return (acc0 + acc1) + (acc2 + acc3);
  }
  int p = p0;
  for (; p + 3 < p1; p += 4) {
    acc0 += src[(long)p * E + e];
    acc1 += src[(long)(p + 1) * E + e];
    acc2 += src[(long)(p + 2) * E + e];
    acc3 += src[(long)(p + 3) * E + e];
  }
  for (; p < p1; ++p) acc0 += src[(long)p * E + e];
  return (acc0 + acc1) + (acc2 + acc3);
}

// out[g][e] = sum_{p in [g*per, min((g+1)*per, P))} in[p][e]   (deterministic)
__global__ void k_reduce_slabs(const float* __restrict__ in, long E, int P, int per, float* __restrict__ out) {
  const long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const int g = blockIdx.y;
  if (e >= E) return;
  const int p0 = g * per, p1 = min(P, p0 + per);
  out[(long)g * E + e] = sum_slab_rows(in, E, e, p0, p1);
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
int theta_to_w_bf16(const float* theta, long theta_stride, int L, int C, const int32_t* w_src, float gamma, void* w,
                    long w_stride, bool balance, hipStream_t s, const int32_t* theta_dst = nullptr,
                    long n_theta = 0);  // (below)

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
    return theta_to_w_bf16(theta, theta_stride, L, C, w_src, gamma, w_out, w_stride, true, s);
  } else {
    return fail(ASR_E_ARG, "asr_theta_to_w: bad dtype %d", dtype);
  }
  return ASR_OK;
}

}  // extern "C"

namespace asr {

// asr_theta_to_w's bf16 pack: balanced rounding (k_theta_to_w_pack_bal) when
// `balance` and C <= 64, round to nearest otherwise (ASR_VARIANT_W_BF16)
int theta_to_w_bf16(const float* theta, long theta_stride, int L, int C, const int32_t* w_src, float gamma, void* w,
                    long w_stride, bool balance, hipStream_t s, const int32_t* theta_dst, long n_theta) {
  const long n = asr_wpack_elems(C);
  if (!theta || !w_src || !w || L < 1 || L > 65535 || n < 0 || w_stride < n)
    return fail(ASR_E_ARG, "theta_to_w_bf16: bad arguments");
  if (balance && (C == 16 || C == 32 || C == 64)) {
    const PackJob job{theta, theta_stride, L, C, w_src, gamma, w, w_stride, theta_dst, n_theta};
    ASR_TRY(theta_to_w_bf16_jobs(&job, 1, s));
  } else {
    const int frags = (C / 16) * ((9 * C + 31) / 32);
    hipLaunchKernelGGL(k_theta_to_w_pack, dim3((frags + 3) / 4, L), dim3(256), 0, s, theta, theta_stride, C, w_src,
                       gamma, (bf16*)w, w_stride);
    ASR_LAUNCH_CHECK("k_theta_to_w_pack");
  }
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
  out[blockIdx.z * out_stride + (long)g * E + e] = sum_slab_rows(src, E, e, p0, p1);
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
