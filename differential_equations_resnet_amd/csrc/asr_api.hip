// C ABI entry points (include/asr.h): conv forward/backward dispatch and the
// native single-block-network executor (stem, L Euler blocks, head, loss,
// backward, Adam).
//
// Reference call stack replaced: Training.train's
// sess.run(train_step) (training/training.py:578-597) over the graph built by
// get_single_block_resnet_build_function (models/tfkeras_resnets.py:547-602)
// and Training._build_optimizer (training/training.py:283-304).
#include <math.h>

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
int reduce_slabs_to_groups(const float* slabs, int P, long ES, float* grp, hipStream_t s);
int reduce_slab_layers(const float* slabs, long slab_stride, int P, long ES, float* grp, long grp_stride, int L,
                       hipStream_t s);
int project_layers(float* grp, long grp_stride, int G, long E, int Cb, const int32_t* theta_dst, long n_theta,
                   int L, float* out, long out_stride, hipStream_t s);
// asr_block_mfma.hip
int block_fwd_mfma(int mode, const void* x, const void* resid, void* y, uint8_t* mask, const void* w,
                   const float* bias, float h, int N, int H, int W, int C, hipStream_t s);
// relu_dx (optional): dx *= [x > 0] when the kernel supports it (*relu_done = 1).
// fold_* (optional): pass 1 of another slab set's reduction (fold_P slabs ->
// reduce_groups(fold_P) group rows at fold_grp), folded into the kernel when
// it supports it (*fold_done = 1); else the caller reduces them itself.
int block_bwd_mfma(int mode, const void* dy, const void* x, const uint8_t* mask, const void* w, float h,
                   float two_gamma, int N, int H, int W, int C, void* dx, float* slabs, int* nslabs, const void* extra,
                   int skip_dy, hipStream_t s, int relu_dx = 0, int* relu_done = nullptr,
                   const float* fold_slabs = nullptr, int fold_P = 0, float* fold_grp = nullptr,
                   int* fold_done = nullptr, int accum = 0);
int stem_wgrad_mfma(const void* img, int input_u8, const void* dz1, int N, int H, int W, int Cin, int C, float mean,
                    float inv_std, int use_norm, float* slabs, int* nslabs, hipStream_t s);
bool stem_wgrad_mfma_supported(int Cin, int H, int W, int C);
int stem_fwd_mfma(const void* img, int input_u8, const float* w1, const float* b1, int N, int H, int W, int Cin, int C,
                  float mean, float inv_std, int use_norm, void* out, hipStream_t s);
bool stem_fwd_mfma_supported(int Cin, int H, int W, int C);
static bool mfma_supported(int C, int W) { return (C == 16 || C == 32 || C == 64) && W == 32; }
// asr_conv_f32.hip: bf16 Euler blocks at any stage width (W in {32, 16, 8}), the multi-stage nets' path
bool convb_supported(int W, int C);
int convb_forward(const void* x, void* y, uint8_t* mask, const void* w, const float* bias, float h, int N, int H, int W,
                  int C, hipStream_t s, bool conv_only = false);
int convb_backward(const void* dy, const uint8_t* mask, const void* x, const void* w, float h, float two_gamma, int N,
                   int H, int W, int C, void* dx, bool need_w, float* slabs, int* nslabs, hipStream_t s,
                   bool conv_only = false);
// asr_deep16.hip
bool deep16_supported(int H, int W, int C);
bool block_stack_fwd_supported(int N, int H, int W, int C);
bool block_stack_bwd_supported(int N, int H, int W, int C);
int block_stack_fwd_rk2_mfma(const void* x0, void* ys, void* xm, long y_stride, uint8_t* masks, uint8_t* masks2,
                             long mask_stride, const void* w, long w_stride, const float* bias, long bias_stride,
                             float h, int N, int H, int W, int C, int L, hipStream_t s);
int block_stack_bwd_grid(int N);
int theta_dst_tile_major(const int32_t* in, long n, int C, int32_t* out, hipStream_t s);
int stack_done_words(int L);
int stack_bwd_reduce_rest(const float* slabs, long slab_stride, int grid, long ES, float* grp, long grp_stride, int L,
                          int lfold, const unsigned* done, hipStream_t s);
int block_stack_bwd_mfma(void* dbuf0, void* dbuf1, const void* xs, long x_stride, const uint8_t* masks,
                         long mask_stride, const void* w, long w_stride, float h, float two_gamma, int N, int H, int W,
                         int C, int L, int ro0, float* slabs, long slab_stride, float* grp, long grp_stride,
                         unsigned* done, int* lfold_out, hipStream_t s, const void* xm = nullptr,
                         const uint8_t* masks2 = nullptr, void* gbuf = nullptr, const void* gtop = nullptr,
                         int fold = 1, int pair = 0);
long stack_slab_floats(int C, int pair);
int theta_dst_pair(const int32_t* in, long n_theta, int C, int32_t* out, hipStream_t s);
int theta_dst_pair_host(const int32_t* in, long n_theta, int C, int32_t* out);
int block_stack_fwd_mfma(const void* x0, void* ys, long y_stride, uint8_t* masks, long mask_stride, const void* w,
                         long w_stride, const float* bias, long bias_stride, float h, int N, int H, int W, int C, int L,
                         hipStream_t s, int slots = 0);
int deep16_forward(const void* x0, void* y0, long y_stride, uint8_t* mask0, long mask_stride, const void* wpack,
                   const float* bias, long bias_stride, float h, int N, int L, bool store_all, hipStream_t s);
int theta_to_w_bf16(const float* theta, long theta_stride, int L, int C, const int32_t* w_src, float gamma, void* w,
                    long w_stride, bool balance, hipStream_t s, const int32_t* theta_dst = nullptr,
                    long n_theta = 0);
size_t deep16_slab_bytes(int N, int L);
int deep16_backward(void* dbufA, void* dbufB, const void* xs, long x_stride, const uint8_t* masks, long mask_stride,
                    const void* wpack, float h, float two_gamma, int N, int L, float* slabs, int* slab_rows,
                    int* dx0_in_b, hipStream_t s);
// asr_conv_f32.hip
int conv_f32(int fmode, const void* xin, void* out, uint8_t* mask, const float* w, const float* bias, float h,
             float two_gamma, const float* dy, int N, int H, int W, int Ci, int Co, int out_bf16, hipStream_t s,
             const float* extra = nullptr);
int make_dz(int fmode, const void* dy, const uint8_t* mask, const void* relu_src, float h, int N, int H, int W, int C,
            int src_bf16, float* dz, hipStream_t s);
int wgrad_f32(const void* x, int x_bf16, const float* dz, int N, int H, int W, int Ci, int Co, float* slabs,
              int* nslabs, hipStream_t s, int K = 3);
int conv_f32_k(int fmode, int K, const void* xin, void* out, uint8_t* mask, const float* w, const float* bias, float h,
               float two_gamma, const float* dy, int N, int H, int W, int C, hipStream_t s, const float* extra);
int wgrad_f32_chunks(int N, int H);
int f32_block_slab_rows(int N, int H, int W, int C);
bool conv32_fused_bwd_supported(int W, int C);
int conv32_bwd_fused(const float* dy, const uint8_t* mask, float h, const float* x, const float* w, float two_gamma,
                     const float* extra, bool skip_dy, int N, int H, int W, int C, float* dx, bool need_w,
                     float* slabs, int* nslabs, hipStream_t s);
// asr_stem_head.hip
bool stem_supported(int Cin, int H, int W, int C);
int stem_forward(const void* img, int input_u8, const float* w1, const float* b1, int N, int H, int W, int Cin, int C,
                 float mean, float inv_std, int use_norm, void* out, int out_bf16, hipStream_t s);
int stem_wgrad(const void* img, int input_u8, const void* dx1, const void* x1, int act_bf16, int N, int H, int W,
               int Cin, int C, float mean, float inv_std, int use_norm, float* slabs, int* nslabs, hipStream_t s);
int head(const void* xL, int act_bf16, const float* fck, const float* fcb, const float* targets, int N, int HW, int C,
         int K, float* probs, float* loss_per, float* dlogits, float* gap, void* dxL, hipStream_t s,
         void* growL = nullptr);
int head_param_grads(const float* gap, const float* dlogits, int N, int C, int K, float* dfck, float* dfcb,
                     const float* loss_per, float* loss_out, hipStream_t s);

constexpr int kMaxSlabsApi = 512;  // matches asr_block_mfma.hip kMaxBlockSlabs
enum { F_EULER = 0, F_CONV = 1, F_RELU = 2, B_EULER = 3, B_CONV = 4 };

static int check_shape(int N, int H, int W, int C) {
  if (N < 1 || H < 1 || W < 1 || C < 1) return fail(ASR_E_ARG, "bad shape N=%d H=%d W=%d C=%d", N, H, W, C);
  if ((long)N * H * W * C > (1L << 40)) return fail(ASR_E_ARG, "shape too large");
  return ASR_OK;
}

// ---------------------------------------------------------------------------
// conv backward workspace
// ---------------------------------------------------------------------------
// `stages` = conv applications whose weight-gradient slabs are reduced
// together (1: Euler block / bare conv, 2: RK2 midpoint block).  RK2 also
// needs the inter-stage gradient g.
struct BwdWs {
  size_t dz, slabs, red, g, total;
};

static BwdWs bwd_ws_layout(int N, int H, int W, int C, int dtype, int stages = 1, int K = 3, int slab_rows = -1) {
  BwdWs b{};
  const long E = (long)K * K * C * C;
  const long P = (long)N * H * W * C;
  const int nsl = slab_rows >= 0 ? slab_rows : kMaxSlabsApi * stages;
  size_t off = 0;
  b.dz = off;
  if (dtype == ASR_F32) off += align_up((size_t)P * 4, 256);
  b.slabs = off;
  off += align_up((size_t)nsl * (E + C) * 4, 256);
  b.red = off;
  off += align_up(reduce_ws_bytes(nsl, E + C), 256);
  b.g = off;
  if (stages > 1) off += align_up((size_t)P * (dtype == ASR_BF16 ? 2 : 4), 256);
  b.total = off;
  return b;
}

// One conv application's backward: dx = [dy] + extra + A^T dz and the
// weight-gradient slabs (written at `slabs`, count in *nsl).
//   EULER: dz = h*dy*mask; CONV: dz = dy.  skip_dy drops the +dy residual of
//   EULER (the second RK2 stage); extra (nullable) is added to dx (the first
//   RK2 stage adds the step's outer dy).
static int block_backward(int mode, const void* dy, const void* x, const uint8_t* mask, const void* w, float h,
                          float gamma, int N, int H, int W, int C, int dtype, void* dx, bool need_w, const void* extra,
                          bool skip_dy, float* slabs, float* dz_scratch, int* nsl, hipStream_t s, bool relu_dx = false,
                          int* relu_done = nullptr, const float* fold_slabs = nullptr, int fold_P = 0,
                          float* fold_grp = nullptr, int* fold_done = nullptr, bool accum_slabs = false) {
  *nsl = 0;
  if (relu_done) *relu_done = 0;
  if (fold_done) *fold_done = 0;
  if (dtype == ASR_BF16) {
    if (!dx && !need_w) return ASR_OK;
    if (!mfma_supported(C, W)) {  // W = 16 / 8: the any-width bf16 kernels (plain Euler blocks and bare convs)
      if (extra || skip_dy || relu_dx || fold_slabs || accum_slabs || !convb_supported(W, C))
        return fail(ASR_E_UNSUPPORTED, "bf16 backward at C=%d W=%d: plain Euler blocks and convs only", C, W);
      return convb_backward(dy, mask, x, w, h, 2.f * gamma, N, H, W, C, dx, need_w, slabs, nsl, s,
                            mode == ASR_MODE_CONV);
    }
    const int cm = (mode == ASR_MODE_EULER) ? 2 : 3;  // BWD_EULER / BWD_CONV
    return block_bwd_mfma(cm, dy, x, mask, w, h, 2.f * gamma, N, H, W, C, dx, slabs, nsl, extra, skip_dy ? 1 : 0, s,
                          relu_dx ? 1 : 0, relu_done, fold_slabs, fold_P, fold_grp, fold_done, accum_slabs ? 1 : 0);
  }
  if (accum_slabs) return fail(ASR_E_UNSUPPORTED, "slab accumulation: bf16 path only");
  const bool euler = mode == ASR_MODE_EULER;
  if (euler && conv32_fused_bwd_supported(W, C))  // fp32 MFMA: dz formed while staging, no dz pass
    return conv32_bwd_fused((const float*)dy, mask, h, (const float*)x, (const float*)w, 2.f * gamma,
                            (const float*)extra, skip_dy, N, H, W, C, (float*)dx, need_w, slabs, nsl, s);
  ASR_TRY(make_dz(euler ? F_EULER : F_CONV, dy, mask, nullptr, h, N, H, W, C, 0, dz_scratch, s));
  if (dx)
    ASR_TRY(conv_f32((euler && !skip_dy) ? B_EULER : B_CONV, dz_scratch, dx, nullptr, (const float*)w, nullptr, h,
                     2.f * gamma, (const float*)dy, N, H, W, C, C, 0, s, (const float*)extra));
  if (need_w) ASR_TRY(wgrad_f32(x, 0, dz_scratch, N, H, W, C, C, slabs, nsl, s));
  return ASR_OK;
}

static int conv_backward_impl(int mode, const void* dy, const void* x, const uint8_t* mask, const void* w,
                              const int32_t* theta_dst, long n_theta, float h, float gamma, int N, int H, int W,
                              int C, int dtype, void* dx, float* dtheta, float* dbias, float* dw_hwio, void* ws,
                              hipStream_t s, float* grp_defer = nullptr, int* nsl_out = nullptr, bool relu_dx = false,
                              int* relu_done = nullptr) {
  const BwdWs L = bwd_ws_layout(N, H, W, C, dtype);
  unsigned char* base = (unsigned char*)ws;
  float* slabs = (float*)(base + L.slabs);
  float* red = (float*)(base + L.red);
  const bool need_w = dtheta || dbias || dw_hwio;
  int nsl = 0;
  ASR_TRY(block_backward(mode, dy, x, mask, w, h, gamma, N, H, W, C, dtype, dx, need_w || grp_defer, nullptr, false,
                         slabs, (float*)(base + L.dz), &nsl, s, relu_dx, relu_done));
  if (grp_defer) {  // the network defers pass 2 + projection to one launch for all layers
    if (nsl_out) *nsl_out = nsl;
    return reduce_slabs_to_groups(slabs, nsl, 9L * C * C + C, grp_defer, s);
  }
  if (need_w)
    ASR_TRY(reduce_and_project(slabs, nsl, 9L * C * C, C, dtheta ? theta_dst : nullptr, n_theta, dtheta, dbias,
                               dw_hwio, red, s));
  return ASR_OK;
}

// One fp32 Euler block's backward that leaves its weight-gradient slabs (*nsl rows of 9C^2 + C
// floats) at `slabs` for the caller to reduce together with other blocks' (reduce_slab_layers).
int conv_backward_keep_slabs(const void* dy, const void* x, const uint8_t* mask, const void* w, float h, float gamma,
                             int N, int H, int W, int C, void* dx, void* ws, float* slabs, int* nsl, hipStream_t s) {
  const BwdWs L = bwd_ws_layout(N, H, W, C, ASR_F32);
  return block_backward(ASR_MODE_EULER, dy, x, mask, w, h, gamma, N, H, W, C, ASR_F32, dx, true, nullptr, false, slabs,
                        (float*)((unsigned char*)ws + L.dz), nsl, s);
}

// RK2 (explicit midpoint) block, BASELINE config 5 (an extension: the
// reference integrates with forward Euler only, tfkeras_resnets.py:69-92):
//   xm = x + (h/2) relu(A x + b)          (mask1 = [A x + b > 0])
//   y  = x + h relu(A xm + b)             (mask2 = [A xm + b > 0])
// Both stages run the Euler kernels; the second takes its residual from x.
static int rk2_forward_impl(const void* x, void* xmid, void* y, uint8_t* mask1, uint8_t* mask2, const void* w,
                            const float* bias, float h, int N, int H, int W, int C, int dtype, hipStream_t s) {
  if (dtype == ASR_BF16) {
    ASR_TRY(block_fwd_mfma(0, x, nullptr, xmid, mask1, w, bias, 0.5f * h, N, H, W, C, s));
    return block_fwd_mfma(0, xmid, x, y, mask2, w, bias, h, N, H, W, C, s);
  }
  ASR_TRY(conv_f32(F_EULER, x, xmid, mask1, (const float*)w, bias, 0.5f * h, 0.f, nullptr, N, H, W, C, C, 0, s));
  return conv_f32(F_EULER, xmid, y, mask2, (const float*)w, bias, h, 0.f, nullptr, N, H, W, C, C, 0, s,
                  (const float*)x);
}

// Backward of rk2_forward_impl: with dz2 = h dy mask2 and g = A^T dz2 (the
// gradient reaching xm), dz1 = (h/2) g mask1 and dx = dy + g + A^T dz1;
// dW collects x (x) dz1 + xm (x) dz2.  bf16: both stages run on the same
// persistent grid, so the first stage adds its slabs onto the second's (one
// slab set per block, *nsl = the grid); fp32: two slab sets, reduced together.
// fold_* as block_bwd_mfma (carried by the second stage's kernel).
static int rk2_backward_slabs(const void* dy, const void* x, const void* xmid, const uint8_t* mask1,
                              const uint8_t* mask2, const void* w, float h, float gamma, int N, int H, int W, int C,
                              int dtype, void* dx, void* g, bool need_w, float* slabs, float* dz_scratch, int* nsl,
                              hipStream_t s, const float* fold_slabs = nullptr, int fold_P = 0,
                              float* fold_grp = nullptr, int* fold_done = nullptr) {
  int n2 = 0, n1 = 0;
  // bf16: both stages run on the same persistent grid (block_bwd_grid of the
  // same shape), so the first stage can add onto the second's slabs
  const bool one_set = dtype == ASR_BF16;
  ASR_TRY(block_backward(ASR_MODE_EULER, dy, xmid, mask2, w, h, gamma, N, H, W, C, dtype, g, need_w, nullptr, true,
                         slabs, dz_scratch, &n2, s, false, nullptr, fold_slabs, fold_P, fold_grp, fold_done));
  ASR_TRY(block_backward(ASR_MODE_EULER, g, x, mask1, w, 0.5f * h, gamma, N, H, W, C, dtype, dx, need_w, dy, false,
                         one_set ? slabs : slabs + (long)n2 * (9L * C * C + C), dz_scratch, &n1, s, false, nullptr,
                         nullptr, 0, nullptr, nullptr, one_set));
  *nsl = one_set ? n2 : n1 + n2;
  return ASR_OK;
}

// ---------------------------------------------------------------------------
// optimizer
// ---------------------------------------------------------------------------
__global__ void k_adam(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                       float* __restrict__ v, long n, float lr_t, float b1, float b2, float eps, float gscale) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float gi = g[i] * gscale;
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    p[i] -= lr_t * mi / (sqrtf(vi) + eps);
  }
}

// dz1 = dx1 * [x1 > 0] in place (bf16, 8 elements per thread): the stem's
// relu' for networks whose first block's backward cannot fuse it (RK2)
__global__ __launch_bounds__(256) void k_relu_grad_bf16(bf16* __restrict__ d, const bf16* __restrict__ x, long n8) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    bf16x8 dv = ((const bf16x8*)d)[i];
    const bf16x8 xv = ((const bf16x8*)x)[i];
#pragma unroll
    for (int e = 0; e < 8; ++e) dv[e] = (float)xv[e] > 0.f ? dv[e] : (bf16)0.f;
    ((bf16x8*)d)[i] = dv;
  }
}

// host: k_relu_grad_bf16 over n elements (n % 8 == 0), in place on d
int relu_grad_bf16(void* d, const void* x, long n, hipStream_t s) {
  if (n % 8) return fail(ASR_E_ARG, "relu_grad_bf16: n %% 8 != 0");
  const long n8 = n / 8;
  hipLaunchKernelGGL(k_relu_grad_bf16, dim3((unsigned)std::max<long>(1, std::min<long>((n8 + 255) / 256, 4096))),
                     dim3(256), 0, s, (bf16*)d, (const bf16*)x, n8);
  ASR_LAUNCH_CHECK("k_relu_grad_bf16");
  return ASR_OK;
}

// ---------------------------------------------------------------------------
// metrics
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_segment_sq_norms(const float* __restrict__ x, const long* __restrict__ off,
                                                          float* __restrict__ out) {
  const long b = off[blockIdx.x], e = off[blockIdx.x + 1];
  float acc = 0.f;
  for (long i = b + threadIdx.x; i < e; i += blockDim.x) acc = fmaf(x[i], x[i], acc);
  for (int d = 32; d >= 1; d >>= 1) acc += __shfl_xor(acc, d, 64);
  __shared__ float part[4];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = (part[0] + part[1]) + (part[2] + part[3]);
}

// loss == nullptr: the batch-mean Keras categorical cross-entropy is computed
// from the probabilities here (evaluation runs forward only).
__global__ __launch_bounds__(256) void k_batch_metrics(const float* __restrict__ probs, const float* __restrict__ tgt,
                                                       const float* __restrict__ loss, int N, int K,
                                                       float* __restrict__ accum) {
  __shared__ int correct;
  __shared__ float lsum[4];
  if (threadIdx.x == 0) correct = 0;
  __syncthreads();
  float l = 0.f;
  for (int n = threadIdx.x; n < N; n += blockDim.x) {
    const float* p = probs + (long)n * K;
    const float* t = tgt + (long)n * K;
    int ap = 0, at = 0;
    float bp = p[0], bt = t[0], s = 0.f;
    for (int k = 0; k < K; ++k) {  // first maximum, as tf.argmax
      if (p[k] > bp) bp = p[k], ap = k;
      if (t[k] > bt) bt = t[k], at = k;
      s += p[k];
    }
    if (ap == at) atomicAdd(&correct, 1);
    if (!loss)
      for (int k = 0; k < K; ++k) {
        const float q = fminf(fmaxf(p[k] / s, 1e-7f), 1.f - 1e-7f);
        l -= t[k] * logf(q);
      }
  }
  for (int d = 32; d >= 1; d >>= 1) l += __shfl_xor(l, d, 64);
  if ((threadIdx.x & 63) == 0) lsum[threadIdx.x >> 6] = l;
  __syncthreads();
  if (threadIdx.x == 0) {
    accum[0] += loss ? *loss : ((lsum[0] + lsum[1]) + (lsum[2] + lsum[3])) / (float)N;
    accum[1] += (float)correct;
    accum[2] += (float)N;
    accum[3] += 1.f;
  }
}

// ---------------------------------------------------------------------------
// network layout
// ---------------------------------------------------------------------------
template <typename Tin>
__global__ void k_normalize(const Tin* __restrict__ img, long n, float mean, float inv_std, int use_norm,
                            float* __restrict__ out) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float v = (float)img[i];
    if (use_norm) v = (v - mean) * inv_std;
    out[i] = v;
  }
}

struct NetLayout {
  long ntheta, P, E, wstride;  // wstride in elements of the W dtype
  long off_c1k, off_c1b, off_blk, blk_stride, off_fck, off_fcb, nparams;
  bool sep_bwd;  // operator not antisymmetric: dgrad uses W_bwd = -flip(W)^T
  bool rk2;      // RK2 midpoint blocks (x_mid activations, two masks per block)
  int stages;    // conv applications per block (1 Euler, 2 RK2)
  long grp_stride;  // floats of slab group sums per layer
  size_t grp;  // per-layer slab group sums, projected after the whole backward
  size_t slabs_all;  // fp32: every block's slabs, pass 1 of all blocks in one launch after the loop
  long slab_stride;
  size_t w_src, w_src_bwd, theta_dst, wbuf, wbuf_bwd, x0, acts, xmids, masks, dxa, dxb, dxg, bwdws, slabs2, slabs, red, probs,
      loss_per, dlogits, gap, total;
  long mask_bytes;
  int act_bytes;
  bool fast_stem;
  bool deep;          // C=16 stack path: one fused launch forward, one backward (asr_deep16.hip)
  size_t deep_slabs;  // its weight-gradient slabs [L][rows][E+C]
  bool inference;     // ASR_VARIANT_INFERENCE: forward-only workspace (3 activation slots, no backward buffers)
  bool stack_bwd;     // C=64 Euler bf16: all blocks' backward in one k_bwd3_stack launch
  bool stack_pair;    // ... with pair-local slabs (antisymmetric operator: the 74 D tiles, not dW)
  int stack_grid;     // its workgroups
  size_t theta_dst_tm, stack_slabs, stack_done;  // tile-major projection map, [L][grid][E+C] slabs, counters
  size_t theta_dst_pr;  // the pull-back from the pair-local slabs (stack_pair)
  int f32_rows;         // fp32: slab rows of one block application's weight gradient (f32_block_slab_rows)
  size_t grow;        // stacked Euler backward: dL/dx_L as one bf16 row per image (the GAP gradient) [N][C]
};

static int net_check(const asr_net_config* c) {
  if (!c) return fail(ASR_E_ARG, "null config");
  ASR_TRY(check_shape(c->N, c->H, c->W, c->C));
  if (c->L < 1 || c->Cin < 1 || c->num_classes < 1 || c->num_classes > 256 || c->C > 256)
    return fail(ASR_E_ARG, "bad net config (L=%d Cin=%d K=%d C=%d)", c->L, c->Cin, c->num_classes, c->C);
  if (c->dtype != ASR_F32 && c->dtype != ASR_BF16) return fail(ASR_E_ARG, "bad dtype");
  if (param_is_antisymmetric(c->param_kind, c->antisymmetric) < 0) return ASR_E_ARG;
  if (c->param_kind == ASR_PARAM_3BY3 && !c->antisymmetric)
    return fail(ASR_E_ARG, "the 3by3 parametrisation is always antisymmetric");
  if (c->integrator != ASR_INTEGRATOR_EULER && c->integrator != ASR_INTEGRATOR_RK2)
    return fail(ASR_E_ARG, "bad integrator %d", c->integrator);
  if (c->variant & ~(ASR_VARIANT_NO_FOLD | ASR_VARIANT_STEM_FWD_VALU | ASR_VARIANT_STEM_WGRAD_VALU | ASR_VARIANT_PER_BLOCK_FWD |
                    ASR_VARIANT_PER_BLOCK_BWD | ASR_VARIANT_INFERENCE | ASR_VARIANT_TIMED | ASR_VARIANT_FULL_DXL |
                    ASR_VARIANT_FULL_SLABS | ASR_VARIANT_W_BF16))
    return fail(ASR_E_ARG, "bad variant bits 0x%x", c->variant);
  if (c->dtype == ASR_BF16 && !mfma_supported(c->C, c->W))
    return fail(ASR_E_UNSUPPORTED, "bf16 network needs C in {16,32,64} and W == 32 (C=%d W=%d)", c->C, c->W);
  return ASR_OK;
}

static NetLayout net_layout(const asr_net_config* c) {
  NetLayout L{};
  const int C = c->C, K = c->num_classes;
  L.ntheta = theta_count(C, c->param_kind, c->antisymmetric);
  L.sep_bwd = param_is_antisymmetric(c->param_kind, c->antisymmetric) == 0;
  L.rk2 = c->integrator == ASR_INTEGRATOR_RK2;
  L.stages = L.rk2 ? 2 : 1;
  L.P = (long)c->N * c->H * c->W * C;
  L.E = 9L * C * C;
  L.act_bytes = c->dtype == ASR_BF16 ? 2 : 4;
  L.wstride = c->dtype == ASR_BF16 ? (long)(C / 16) * ((9 * C + 31) / 32) * 512 : L.E;
  L.off_c1k = 0;
  L.off_c1b = 9L * c->Cin * C;
  L.off_blk = L.off_c1b + C;
  L.blk_stride = L.ntheta + C;
  L.off_fck = L.off_blk + (long)c->L * L.blk_stride;
  L.off_fcb = L.off_fck + (long)C * K;
  L.nparams = L.off_fcb + K;
  L.mask_bytes = asr_mask_bytes(c->N, c->H, c->W, C);
  L.fast_stem = stem_supported(c->Cin, c->H, c->W, C);
  L.inference = (c->variant & ASR_VARIANT_INFERENCE) != 0;
  const bool tr = !L.inference;  // training buffers
  L.deep = c->dtype == ASR_BF16 && !L.rk2 && deep16_supported(c->H, c->W, C);
  L.stack_bwd = tr && c->dtype == ASR_BF16 && block_stack_bwd_supported(c->N, c->H, c->W, C);
  L.stack_grid = L.stack_bwd ? block_stack_bwd_grid(c->N) : 0;
  L.stack_pair = L.stack_bwd && !L.sep_bwd;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off += align_up(bytes, 256);
    return o;
  };
  L.w_src = take((size_t)L.E * 4);
  L.w_src_bwd = take(L.sep_bwd && tr ? (size_t)L.E * 4 : 0);
  L.theta_dst = take((size_t)L.ntheta * 2 * 4);
  L.wbuf = take((size_t)c->L * L.wstride * L.act_bytes);
  L.wbuf_bwd = take(L.sep_bwd && tr ? (size_t)c->L * L.wstride * L.act_bytes : 0);
  L.x0 = take(L.fast_stem ? 0 : (size_t)c->N * c->H * c->W * c->Cin * 4);
  // training keeps x_0 .. x_L for the backward; inference ping-pongs (x_0 + 2 slots)
  L.acts = take((size_t)(tr ? c->L + 1 : 3) * L.P * L.act_bytes);
  L.xmids = take(L.rk2 ? (size_t)(tr ? c->L : 1) * L.P * L.act_bytes : 0);
  L.masks = take(tr ? (size_t)L.stages * c->L * L.mask_bytes : 0);  // RK2: mask1 of every block, then mask2
  L.dxa = take(tr ? (size_t)L.P * L.act_bytes : 0);
  L.dxb = take(tr ? (size_t)L.P * L.act_bytes : 0);
  L.dxg = take(L.rk2 && tr ? (size_t)L.P * L.act_bytes : 0);
  // per-block backward workspace (asr_conv_backward layout), reused by the stem.
  // fp32 keeps every block's slabs in slabs_all, sized by the grid its weight
  // gradient runs (not the 512-row maximum): no slab rows here, no slabs2
  const bool f32 = c->dtype == ASR_F32;
  L.f32_rows = f32 ? f32_block_slab_rows(c->N, c->H, c->W, C) : 0;
  const BwdWs bw = bwd_ws_layout(c->N, c->H, c->W, C, c->dtype, L.stages, 3, f32 ? 0 : -1);
  const long E1 = 9L * c->Cin * C;
  const size_t stem_ws = align_up((size_t)L.P * 4, 256) + align_up((size_t)kMaxSlabsApi * (E1 + C) * 4, 256) +
                         align_up(reduce_ws_bytes(kMaxSlabsApi, E1 + C), 256);
  L.bwdws = take(tr ? std::max(bw.total, stem_ws) : 0);
  // odd Euler blocks' slabs (even ones use the backward workspace's): a
  // block's slabs stay readable while the next block's kernel reduces them
  L.slabs2 = take(tr && !f32 ? (size_t)L.stages * kMaxSlabsApi * (L.E + C) * 4 : 0);  // every other block's slabs
  const int rows = f32 ? L.stages * L.f32_rows : L.stages * kMaxSlabsApi;
  L.grp_stride = (long)reduce_groups(rows) * (L.E + C);
  L.grp = take(tr ? (size_t)c->L * L.grp_stride * 4 : 0);
  L.slab_stride = (long)rows * (L.E + C);
  L.slabs_all = take(tr && f32 ? (size_t)c->L * L.slab_stride * 4 : 0);
  L.deep_slabs = take(L.deep && tr ? deep16_slab_bytes(c->N, c->L) : 0);
  L.theta_dst_tm = take(L.stack_bwd ? (size_t)L.ntheta * 2 * 4 : 0);
  L.theta_dst_pr = take(L.stack_pair ? (size_t)L.ntheta * 2 * 4 : 0);
  L.stack_slabs = take(L.stack_bwd ? (size_t)c->L * L.stack_grid * (L.E + C) * 4 : 0);
  L.stack_done = take(L.stack_bwd ? (size_t)stack_done_words(c->L) * 4 : 0);
  L.grow = take(L.stack_bwd && !L.rk2 ? (size_t)c->N * C * 2 : 0);
  L.probs = take((size_t)c->N * K * 4);
  L.loss_per = take(tr ? (size_t)c->N * 4 : 0);
  L.dlogits = take(tr ? (size_t)c->N * K * 4 : 0);
  L.gap = take(tr ? (size_t)c->N * C * 4 : 0);
  L.total = off;
  return L;
}

// ASR_VARIANT_TIMED: HIP events around the block launches of the last timed
// asr_net_forward / asr_net_forward_backward (asr_net_kernel_times): 0-1 the
// blocks' forward, 2-3 the stacked backward kernel, 3-4 its post-launch slab
// reductions and the projection onto theta.  Measurement only.  The events are
// kept per device (created on that device at its first timed call); on one
// device, timed calls from several host threads at once overwrite each
// other's times (one timing thread per device).
constexpr int kMaxTimedDevices = 64;
struct TimedEvents {
  hipEvent_t ev[5];
  bool made;
  unsigned rec;  // bit i: event i recorded by the last timed call on this device
};
static TimedEvents g_tev[kMaxTimedDevices];

static TimedEvents* timed_events_here() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxTimedDevices) return nullptr;
  return &g_tev[dev];
}

static int timed_event(const asr_net_config* c, int i, hipStream_t s) {
  if (!(c->variant & ASR_VARIANT_TIMED)) return ASR_OK;
  TimedEvents* t = timed_events_here();
  if (!t) return fail(ASR_E_HIP, "ASR_VARIANT_TIMED: no current device (or device id >= %d)", kMaxTimedDevices);
  if (!t->made) {
    for (auto& e : t->ev) ASR_TRY(hip_check(hipEventCreate(&e), "hipEventCreate"));
    t->made = true;
  }
  if (i == 0) t->rec = 0;
  ASR_TRY(hip_check(hipEventRecord(t->ev[i], s), "hipEventRecord"));
  t->rec |= 1u << i;
  return ASR_OK;
}

// x_L of a forward: training keeps every activation (slot L); evaluation
// ping-pongs (the C=64 stack over slots 1-2 of the inference layout, the
// per-block kernels over slots 0-1)
static unsigned char* net_xL(const asr_net_config* c, const NetLayout& L, unsigned char* ws, bool training,
                             bool stack_fwd) {
  const size_t a = (size_t)L.P * L.act_bytes;
  if (training) return ws + L.acts + (size_t)c->L * a;
  if (stack_fwd) return ws + L.acts + (size_t)(1 + (c->L - 1) % 2) * a;
  return ws + L.acts + (size_t)(c->L & 1) * a;
}

static int net_forward_impl(const asr_net_config* c, const NetLayout& L, const float* params, const void* images,
                            bool training, unsigned char* ws, hipStream_t s, unsigned char** xL_out = nullptr) {
  const int C = c->C, N = c->N, H = c->H, W = c->W;
  const bool bf = c->dtype == ASR_BF16;
  const float inv_std = c->use_norm ? 1.f / c->divide_by_stddev : 1.f;
  if (training && L.inference) return fail(ASR_E_ARG, "an ASR_VARIANT_INFERENCE workspace has no training buffers");
  // 1. materialise W for all L blocks (one launch)
  //    (bf16: balanced rounding of the antisymmetric pairs, k_theta_to_w_pack_bal; ASR_VARIANT_W_BF16: to nearest)
  const bool bal = !(c->variant & ASR_VARIANT_W_BF16);
  if (bf)
    ASR_TRY(theta_to_w_bf16(params + L.off_blk, L.blk_stride, c->L, C, (const int32_t*)(ws + L.w_src), c->gamma,
                            ws + L.wbuf, L.wstride, bal, s,
                            c->param_kind != ASR_PARAM_REGULAR ? (const int32_t*)(ws + L.theta_dst) : nullptr,
                            L.ntheta));
  else
    ASR_TRY(asr_theta_to_w(params + L.off_blk, L.blk_stride, c->L, C, (const int32_t*)(ws + L.w_src), c->gamma,
                           ws + L.wbuf, L.wstride, c->dtype, s));
  if (training && L.sep_bwd) {  // (the transposed map pairs the same entries: W_bwd = -W^T after the rounding too)
    if (bf)
      ASR_TRY(theta_to_w_bf16(params + L.off_blk, L.blk_stride, c->L, C, (const int32_t*)(ws + L.w_src_bwd), 0.f,
                              ws + L.wbuf_bwd, L.wstride, bal, s));
    else
      ASR_TRY(asr_theta_to_w(params + L.off_blk, L.blk_stride, c->L, C, (const int32_t*)(ws + L.w_src_bwd), 0.f,
                             ws + L.wbuf_bwd, L.wstride, c->dtype, s));
  }
  unsigned char* acts = ws + L.acts;
  auto act = [&](int i) -> unsigned char* {
    const int slot = training ? i : (i & 1);
    return acts + (size_t)slot * L.P * L.act_bytes;
  };
  if (xL_out) *xL_out = net_xL(c, L, ws, training, false);
  // 2. normalisation + conv1 + relu (tfkeras_resnets.py:555-572)
  if (L.fast_stem && bf && stem_fwd_mfma_supported(c->Cin, H, W, C) && !(c->variant & ASR_VARIANT_STEM_FWD_VALU)) {
    ASR_TRY(stem_fwd_mfma(images, c->input_u8, params + L.off_c1k, params + L.off_c1b, N, H, W, c->Cin, C,
                          c->subtract_mean, inv_std, c->use_norm, act(0), s));
  } else if (L.fast_stem) {
    ASR_TRY(stem_forward(images, c->input_u8, params + L.off_c1k, params + L.off_c1b, N, H, W, c->Cin, C,
                         c->subtract_mean, inv_std, c->use_norm, act(0), bf ? 1 : 0, s));
  } else {
    const long nin = (long)N * H * W * c->Cin;
    float* x0 = (float*)(ws + L.x0);
    const unsigned gn = (unsigned)std::min<long>((nin + 255) / 256, 4096);
    if (c->input_u8)
      hipLaunchKernelGGL(k_normalize<uint8_t>, dim3(gn), dim3(256), 0, s, (const uint8_t*)images, nin,
                         c->subtract_mean, inv_std, c->use_norm, x0);
    else
      hipLaunchKernelGGL(k_normalize<float>, dim3(gn), dim3(256), 0, s, (const float*)images, nin,
                         c->subtract_mean, inv_std, c->use_norm, x0);
    ASR_LAUNCH_CHECK("k_normalize");
    ASR_TRY(conv_f32(F_RELU, x0, act(0), nullptr, params + L.off_c1k, params + L.off_c1b, 1.f, 0.f, nullptr, N, H,
                     W, c->Cin, C, bf ? 1 : 0, s));
  }
  // 3. L Euler blocks (tfkeras_resnets.py:579-582 -> :28-94), or RK2 blocks
  ASR_TRY(timed_event(c, 0, s));
  if (L.deep) {  // C=16: all L steps in one launch, images resident in LDS
    ASR_TRY(deep16_forward(act(0), act(training ? 1 : c->L), L.P, training ? (uint8_t*)(ws + L.masks) : nullptr,
                           L.mask_bytes, ws + L.wbuf, params + L.off_blk + L.ntheta, L.blk_stride, c->h, N, c->L,
                           training, s));
    return timed_event(c, 1, s);
  }
  if (bf && training && L.rk2 && block_stack_fwd_supported(N, H, W, C) && !(c->variant & ASR_VARIANT_PER_BLOCK_FWD)) {
    // C=64 RK2: all 2L stages in one launch
    uint8_t* m1 = (uint8_t*)(ws + L.masks);
    ASR_TRY(block_stack_fwd_rk2_mfma(act(0), act(1), ws + L.xmids, (long)L.P, m1, m1 + (size_t)c->L * L.mask_bytes,
                                     (long)L.mask_bytes, ws + L.wbuf, (long)L.wstride, params + L.off_blk + L.ntheta,
                                     L.blk_stride, c->h, N, H, W, C, c->L, s));
    return timed_event(c, 1, s);
  }
  if (bf && !L.rk2 && (training || L.inference) && block_stack_fwd_supported(N, H, W, C) &&
      !(c->variant & ASR_VARIANT_PER_BLOCK_FWD)) {
    // C=64: all L blocks in one launch (whole images per workgroup); inference
    // ping-pongs x_l between slots 1 and 2 with no relu masks
    if (training) {
      ASR_TRY(block_stack_fwd_mfma(act(0), act(1), (long)L.P, (uint8_t*)(ws + L.masks), (long)L.mask_bytes,
                                   ws + L.wbuf, (long)L.wstride, params + L.off_blk + L.ntheta, L.blk_stride, c->h, N,
                                   H, W, C, c->L, s));
    } else {
      ASR_TRY(block_stack_fwd_mfma(acts, acts + (size_t)L.P * L.act_bytes, (long)L.P, nullptr, 0, ws + L.wbuf,
                                   (long)L.wstride, params + L.off_blk + L.ntheta, L.blk_stride, c->h, N, H, W, C,
                                   c->L, s, 2));
      if (xL_out) *xL_out = net_xL(c, L, ws, false, true);
    }
    return timed_event(c, 1, s);
  }
  for (int l = 0; l < c->L; ++l) {
    const float* bias = params + L.off_blk + (long)l * L.blk_stride + L.ntheta;
    const unsigned char* wl = ws + L.wbuf + (size_t)l * L.wstride * L.act_bytes;
    uint8_t* mask = training ? (uint8_t*)(ws + L.masks) + (size_t)l * L.mask_bytes : nullptr;
    if (L.rk2) {
      unsigned char* xm = ws + L.xmids + (training ? (size_t)l * L.P * L.act_bytes : 0);
      uint8_t* mask2 = training ? mask + (size_t)c->L * L.mask_bytes : nullptr;
      ASR_TRY(rk2_forward_impl(act(l), xm, act(l + 1), mask, mask2, wl, bias, c->h, N, H, W, C, c->dtype, s));
    } else if (bf) {
      ASR_TRY(block_fwd_mfma(0, act(l), nullptr, act(l + 1), mask, wl, bias, c->h, N, H, W, C, s));
    } else {
      ASR_TRY(conv_f32(F_EULER, act(l), act(l + 1), mask, (const float*)wl, bias, c->h, 0.f, nullptr, N, H, W, C, C,
                       0, s));
    }
  }
  return timed_event(c, 1, s);
}

}  // namespace asr

using namespace asr;

extern "C" {

long asr_mask_bytes(int N, int H, int W, int C) {
  if (N < 1 || H < 1 || W < 1 || C < 1) return -1;
  return ((long)N * H * W * C + 31) / 32 * 4;
}

int asr_conv_forward(int mode, const void* x, void* y, uint8_t* mask, const void* w, const float* bias, float h,
                     int N, int H, int W, int C, int dtype, asr_stream_t stream) {
  ASR_TRY(check_shape(N, H, W, C));
  if (!x || !y || !w) return fail(ASR_E_ARG, "asr_conv_forward: null pointer");
  if (mode != ASR_MODE_EULER && mode != ASR_MODE_CONV) return fail(ASR_E_ARG, "asr_conv_forward: bad mode %d", mode);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == ASR_BF16) {
    if (!mfma_supported(C, W)) {  // W = 16 / 8 (multi-stage nets): the any-width bf16 kernels, Euler block or bare conv
      if (convb_supported(W, C))
        return convb_forward(x, y, mask, w, bias, h, N, H, W, C, s, mode == ASR_MODE_CONV);
      return fail(ASR_E_UNSUPPORTED, "bf16 conv needs C in {16,32,64} and W in {32, 16, 8} (C=%d W=%d)", C, W);
    }
    if (mode == ASR_MODE_EULER && deep16_supported(H, W, C))
      return deep16_forward(x, y, 0, mask, 0, w, bias, 0, h, N, 1, true, s);
    return block_fwd_mfma(mode == ASR_MODE_EULER ? 0 : 1, x, nullptr, y, mask, w, bias, h, N, H, W, C, s);
  }
  if (dtype == ASR_F32)
    return conv_f32(mode == ASR_MODE_EULER ? F_EULER : F_CONV, x, y, mask, (const float*)w, bias, h, 0.f, nullptr, N,
                    H, W, C, C, 0, s);
  return fail(ASR_E_ARG, "asr_conv_forward: bad dtype %d", dtype);
}

int asr_block_stack_forward(const void* x0, void* ys, long y_stride, uint8_t* masks, long mask_stride, const void* w,
                            long w_stride, const float* bias, long bias_stride, float h, int N, int H, int W, int C,
                            int L, int dtype, int store_all, asr_stream_t stream) {
  ASR_TRY(check_shape(N, H, W, C));
  if (!x0 || !ys || !w || L < 1) return fail(ASR_E_ARG, "asr_block_stack_forward: null pointer or L < 1");
  if (store_all && L > 1 && y_stride < (long)N * H * W * C)
    return fail(ASR_E_ARG, "asr_block_stack_forward: y_stride smaller than one activation");
  hipStream_t s = (hipStream_t)stream;
  if (dtype == ASR_BF16 && deep16_supported(H, W, C)) {
    if (L > 1 && w_stride != (long)asr_wpack_elems(C))
      return fail(ASR_E_ARG, "asr_block_stack_forward: w_stride must be asr_wpack_elems(C) on the fused path");
    return deep16_forward(x0, ys, y_stride, masks, mask_stride, w, bias, bias_stride, h, N, L, store_all != 0, s);
  }
  if (dtype == ASR_BF16 && !mfma_supported(C, W))
    return fail(ASR_E_UNSUPPORTED, "bf16 conv needs C in {16,32,64} and W == 32 (C=%d W=%d)", C, W);
  if (dtype != ASR_F32 && dtype != ASR_BF16) return fail(ASR_E_ARG, "asr_block_stack_forward: bad dtype");
  const size_t es = dtype == ASR_BF16 ? 2 : 4;
  if (!store_all && L > 1) return fail(ASR_E_UNSUPPORTED, "asr_block_stack_forward: store_all=0 needs the fused path");
  if (dtype == ASR_BF16 && block_stack_fwd_supported(N, H, W, C))
    return block_stack_fwd_mfma(x0, ys, L > 1 ? y_stride : (long)N * H * W * C, masks, mask_stride, w, w_stride, bias,
                                bias_stride, h, N, H, W, C, L, s);
  for (int l = 0; l < L; ++l) {
    const void* xi = l == 0 ? x0 : (const unsigned char*)ys + (size_t)(l - 1) * y_stride * es;
    void* yo = (unsigned char*)ys + (size_t)l * y_stride * es;
    ASR_TRY(asr_conv_forward(ASR_MODE_EULER, xi, yo, masks ? masks + (size_t)l * mask_stride : nullptr,
                             (const unsigned char*)w + (size_t)l * w_stride * es, bias ? bias + l * bias_stride : nullptr,
                             h, N, H, W, C, dtype, stream));
  }
  return ASR_OK;
}

// workspace of asr_block_stack_backward: two dx buffers, then either the
// fused path's slabs + group rows or one per-block backward workspace
struct StackWs {
  size_t da, db, slabs, grp, blk, done, tdst, g, total;
  bool deep, stack64;
  int grid;
};
static StackWs stack_ws_layout(int N, int H, int W, int C, int L, int dtype, bool rk2 = false) {
  StackWs w{};
  const size_t act = align_up((size_t)N * H * W * C * (dtype == ASR_BF16 ? 2 : 4), 256);
  const long ES = 9L * C * C + C;
  w.deep = !rk2 && dtype == ASR_BF16 && deep16_supported(H, W, C);
  w.stack64 = dtype == ASR_BF16 && !w.deep && block_stack_bwd_supported(N, H, W, C);
  w.grid = w.stack64 ? block_stack_bwd_grid(N) : 0;
  size_t off = 0;
  w.da = off;
  off += act;
  w.db = off;
  off += act;
  if (w.deep) {
    w.slabs = off;
    off += align_up(deep16_slab_bytes(N, L), 256);
    w.grp = off;
    off += align_up((size_t)L * reduce_groups(kMaxSlabsApi) * ES * 4, 256);
  } else if (w.stack64) {  // slabs [L][grid][ES] (tile-major dW), group rows, counters, tile-major theta map
    w.slabs = off;
    off += align_up((size_t)L * w.grid * ES * 4, 256);
    w.grp = off;
    off += align_up((size_t)L * reduce_groups(w.grid) * ES * 4, 256);
    w.done = off;
    off += align_up((size_t)stack_done_words(L) * 4, 256);
    w.tdst = off;
    off += align_up((size_t)2 * 9 * C * C * 4, 256);
    if (rk2) {  // the gradient reaching x_mid between a block's two stages
      w.g = off;
      off += act;
    }
  } else {
    w.blk = off;
    off += bwd_ws_layout(N, H, W, C, dtype).total;
  }
  w.total = off;
  return w;
}

size_t asr_block_stack_backward_workspace_bytes(int N, int H, int W, int C, int L, int dtype) {
  if (check_shape(N, H, W, C) != ASR_OK || L < 1) return 0;
  return stack_ws_layout(N, H, W, C, L, dtype).total;
}

int asr_block_stack_backward(const void* dyL, const void* xs, long x_stride, const uint8_t* masks, long mask_stride,
                             const void* w, long w_stride, const int32_t* theta_dst, long n_theta, float h,
                             float gamma, int N, int H, int W, int C, int L, int dtype, void* dx0, float* dparams,
                             void* ws, size_t ws_bytes, asr_stream_t stream) {
  ASR_TRY(check_shape(N, H, W, C));
  if (!dyL || !xs || !masks || !w || !dx0 || L < 1) return fail(ASR_E_ARG, "asr_block_stack_backward: null pointer");
  if (dparams && !theta_dst) return fail(ASR_E_ARG, "asr_block_stack_backward: theta_dst needed for dparams");
  if (dtype != ASR_F32 && dtype != ASR_BF16) return fail(ASR_E_ARG, "asr_block_stack_backward: bad dtype");
  if (dtype == ASR_BF16 && !mfma_supported(C, W))
    return fail(ASR_E_UNSUPPORTED, "bf16 conv needs C in {16,32,64} and W == 32 (C=%d W=%d)", C, W);
  const StackWs Lw = stack_ws_layout(N, H, W, C, L, dtype);
  if (!ws || ws_bytes < Lw.total) return fail(ASR_E_WORKSPACE, "asr_block_stack_backward: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  unsigned char* base = (unsigned char*)ws;
  const size_t es = dtype == ASR_BF16 ? 2 : 4, act = (size_t)N * H * W * C * es;
  const long E = 9L * C * C;
  if (Lw.deep) {
    if (w_stride != (long)asr_wpack_elems(C))
      return fail(ASR_E_ARG, "asr_block_stack_backward: w_stride must be asr_wpack_elems(C) on the fused path");
    ASR_TRY(hip_check(hipMemcpyAsync(base + Lw.da, dyL, act, hipMemcpyDeviceToDevice, s), "hipMemcpyAsync"));
    int rows = 0, in_b = 0;
    float* slabs = (float*)(base + Lw.slabs);
    ASR_TRY(deep16_backward(base + Lw.da, base + Lw.db, xs, x_stride, masks, mask_stride, w, h, 2.f * gamma, N, L,
                            slabs, &rows, &in_b, s));
    ASR_TRY(hip_check(hipMemcpyAsync(dx0, base + (in_b ? Lw.db : Lw.da), act, hipMemcpyDeviceToDevice, s),
                      "hipMemcpyAsync"));
    if (dparams) {
      const int G = reduce_groups(rows);
      ASR_TRY(reduce_slabs_to_groups(slabs, L * rows, E + C, (float*)(base + Lw.grp), s));
      ASR_TRY(project_layers((float*)(base + Lw.grp), (long)G * (E + C), G, E, C, theta_dst, n_theta, L, dparams,
                             n_theta + C, s));
    }
    return ASR_OK;
  }
  if (Lw.stack64) {
    if (n_theta > 9L * C * C) return fail(ASR_E_ARG, "asr_block_stack_backward: n_theta > 9*C*C");
    ASR_TRY(hip_check(hipMemcpyAsync(base + Lw.da, dyL, act, hipMemcpyDeviceToDevice, s), "hipMemcpyAsync"));
    float* slabs = (float*)(base + Lw.slabs);
    float* grp = (float*)(base + Lw.grp);
    // the stack ABI's operator is antisymmetric (its dgrad is A^T = -A + 2 gamma I): pair-local slabs
    const long ES = stack_slab_floats(C, 1), sst = (long)Lw.grid * ES, gst = (long)reduce_groups(Lw.grid) * ES;
    int lfold = L;
    ASR_TRY(block_stack_bwd_mfma(base + Lw.da, base + Lw.db, xs, x_stride, masks, mask_stride, w, w_stride, h,
                                 2.f * gamma, N, H, W, C, L, 0, slabs, sst, grp, gst, (unsigned*)(base + Lw.done),
                                 &lfold, s, nullptr, nullptr, nullptr, nullptr, 1, 1));
    ASR_TRY(hip_check(hipMemcpyAsync(dx0, base + ((L & 1) ? Lw.db : Lw.da), act, hipMemcpyDeviceToDevice, s),
                      "hipMemcpyAsync"));
    if (dparams) {
      ASR_TRY(stack_bwd_reduce_rest(slabs, sst, Lw.grid, ES, grp, gst, L, lfold, (const unsigned*)(base + Lw.done), s));
      int32_t* tm = (int32_t*)(base + Lw.tdst);
      ASR_TRY(theta_dst_pair(theta_dst, n_theta, C, tm, s));
      ASR_TRY(project_layers(grp, gst, reduce_groups(Lw.grid), ES - C, C, tm, n_theta, L, dparams, n_theta + C, s));
    }
    return ASR_OK;
  }
  // per-block kernels, last block first
  const void* dcur = dyL;
  for (int l = L - 1; l >= 0; --l) {
    void* dnext = l == 0 ? dx0 : base + ((l & 1) ? Lw.db : Lw.da);
    float* dp = dparams ? dparams + (long)l * (n_theta + C) : nullptr;
    ASR_TRY(conv_backward_impl(ASR_MODE_EULER, dcur, (const unsigned char*)xs + (size_t)l * x_stride * es,
                               masks + (size_t)l * mask_stride, (const unsigned char*)w + (size_t)l * w_stride * es,
                               theta_dst, n_theta, h, gamma, N, H, W, C, dtype, dnext, dp, dp ? dp + n_theta : nullptr,
                               nullptr, base + Lw.blk, s));
    dcur = dnext;
  }
  return ASR_OK;
}

int asr_rk2_stack_forward(const void* x0, void* ys, void* xmids, long y_stride, uint8_t* masks1, uint8_t* masks2,
                          long mask_stride, const void* w, long w_stride, const float* bias, long bias_stride, float h,
                          int N, int H, int W, int C, int L, int dtype, asr_stream_t stream) {
  ASR_TRY(check_shape(N, H, W, C));
  if (!x0 || !ys || !xmids || !w || L < 1) return fail(ASR_E_ARG, "asr_rk2_stack_forward: null pointer or L < 1");
  if (dtype != ASR_BF16 || !block_stack_fwd_supported(N, H, W, C))
    return fail(ASR_E_UNSUPPORTED, "asr_rk2_stack_forward: bf16, C=64, W=32 only (C=%d W=%d)", C, W);
  if ((masks1 == nullptr) != (masks2 == nullptr)) return fail(ASR_E_ARG, "asr_rk2_stack_forward: masks1/masks2");
  return block_stack_fwd_rk2_mfma(x0, ys, xmids, y_stride, masks1, masks2, mask_stride, w, w_stride, bias,
                                  bias_stride, h, N, H, W, C, L, (hipStream_t)stream);
}

size_t asr_rk2_stack_backward_workspace_bytes(int N, int H, int W, int C, int L, int dtype) {
  if (check_shape(N, H, W, C) != ASR_OK || L < 1) return 0;
  const StackWs w = stack_ws_layout(N, H, W, C, L, dtype, true);
  return w.stack64 ? w.total : 0;
}

int asr_rk2_stack_backward(const void* dyL, const void* xs, const void* xmids, long x_stride, const uint8_t* masks1,
                           const uint8_t* masks2, long mask_stride, const void* w, long w_stride,
                           const int32_t* theta_dst, long n_theta, float h, float gamma, int N, int H, int W, int C,
                           int L, int dtype, void* dx0, float* dparams, void* ws, size_t ws_bytes,
                           asr_stream_t stream) {
  ASR_TRY(check_shape(N, H, W, C));
  if (!dyL || !xs || !xmids || !masks1 || !masks2 || !w || !dx0 || L < 1)
    return fail(ASR_E_ARG, "asr_rk2_stack_backward: null pointer");
  if (dparams && !theta_dst) return fail(ASR_E_ARG, "asr_rk2_stack_backward: theta_dst needed for dparams");
  const StackWs Lw = stack_ws_layout(N, H, W, C, L, dtype, true);
  if (!Lw.stack64) return fail(ASR_E_UNSUPPORTED, "asr_rk2_stack_backward: bf16, C=64, W=32 only (C=%d W=%d)", C, W);
  if (!ws || ws_bytes < Lw.total) return fail(ASR_E_WORKSPACE, "asr_rk2_stack_backward: workspace too small");
  if (n_theta > 9L * C * C) return fail(ASR_E_ARG, "asr_rk2_stack_backward: n_theta > 9*C*C");
  hipStream_t s = (hipStream_t)stream;
  unsigned char* base = (unsigned char*)ws;
  const size_t act = (size_t)N * H * W * C * 2;
  const long ES = stack_slab_floats(C, 1), sst = (long)Lw.grid * ES, gst = (long)reduce_groups(Lw.grid) * ES;
  ASR_TRY(hip_check(hipMemcpyAsync(base + Lw.da, dyL, act, hipMemcpyDeviceToDevice, s), "hipMemcpyAsync"));
  float* slabs = (float*)(base + Lw.slabs);
  float* grp = (float*)(base + Lw.grp);
  int lfold = L;
  ASR_TRY(block_stack_bwd_mfma(base + Lw.da, base + Lw.db, xs, x_stride, masks1, mask_stride, w, w_stride, h,
                               2.f * gamma, N, H, W, C, L, 0, slabs, sst, grp, gst, (unsigned*)(base + Lw.done),
                               &lfold, s, xmids, masks2, base + Lw.g, nullptr, 1, 1));
  ASR_TRY(hip_check(hipMemcpyAsync(dx0, base + ((L & 1) ? Lw.db : Lw.da), act, hipMemcpyDeviceToDevice, s),
                    "hipMemcpyAsync"));
  if (dparams) {
    ASR_TRY(stack_bwd_reduce_rest(slabs, sst, Lw.grid, ES, grp, gst, L, lfold, (const unsigned*)(base + Lw.done), s));
    int32_t* tm = (int32_t*)(base + Lw.tdst);
    ASR_TRY(theta_dst_pair(theta_dst, n_theta, C, tm, s));
    ASR_TRY(project_layers(grp, gst, reduce_groups(Lw.grid), ES - C, C, tm, n_theta, L, dparams, n_theta + C, s));
  }
  return ASR_OK;
}

size_t asr_conv_backward_workspace_bytes_k(int N, int H, int W, int C, int kernel_size) {
  if (check_shape(N, H, W, C) != ASR_OK || kernel_size < 1 || !(kernel_size & 1)) return 0;
  return bwd_ws_layout(N, H, W, C, ASR_F32, 1, kernel_size).total;
}

// Conv2DAntisymmetric(kernel_size != 3) (…Conv2DAntisymmetric.py:60-68, 109-145, 163-170): the
// same operator family on a K x K kernel, fp32 (the reference's precision) on the VALU kernels;
// K = 3 is asr_conv_forward / asr_conv_backward.
int asr_conv_forward_k(int mode, int kernel_size, const float* x, float* y, uint8_t* mask, const float* w,
                       const float* bias, float h, int N, int H, int W, int C, asr_stream_t stream) {
  ASR_TRY(check_shape(N, H, W, C));
  if (!x || !y || !w) return fail(ASR_E_ARG, "asr_conv_forward_k: null pointer");
  if (mode != ASR_MODE_EULER && mode != ASR_MODE_CONV) return fail(ASR_E_ARG, "asr_conv_forward_k: bad mode %d", mode);
  if (kernel_size < 1 || kernel_size > 15 || !(kernel_size & 1))
    return fail(ASR_E_ARG, "asr_conv_forward_k: kernel_size %d (odd, 1..15)", kernel_size);
  return conv_f32_k(mode == ASR_MODE_EULER ? F_EULER : F_CONV, kernel_size, x, y, mask, w, bias, h, 0.f, nullptr, N, H, W,
                    C, (hipStream_t)stream, nullptr);
}

int asr_conv_backward_k(int mode, int kernel_size, const float* dy, const float* x, const uint8_t* mask,
                        const float* w, const int32_t* theta_dst, long n_theta, float h, float gamma, int N, int H,
                        int W, int C, float* dx, float* dtheta, float* dbias, float* dw, void* ws, size_t ws_bytes,
                        asr_stream_t stream) {
  ASR_TRY(check_shape(N, H, W, C));
  if (mode != ASR_MODE_EULER && mode != ASR_MODE_CONV) return fail(ASR_E_ARG, "asr_conv_backward_k: bad mode %d", mode);
  if (kernel_size < 1 || kernel_size > 15 || !(kernel_size & 1))
    return fail(ASR_E_ARG, "asr_conv_backward_k: kernel_size %d (odd, 1..15)", kernel_size);
  if (!dy || !w || (mode == ASR_MODE_EULER && !mask)) return fail(ASR_E_ARG, "asr_conv_backward_k: null pointer");
  if ((dtheta || dbias || dw) && !x) return fail(ASR_E_ARG, "asr_conv_backward_k: x needed for weight gradients");
  if (dtheta && !theta_dst) return fail(ASR_E_ARG, "asr_conv_backward_k: theta_dst needed for dtheta");
  const BwdWs Lw = bwd_ws_layout(N, H, W, C, ASR_F32, 1, kernel_size);
  if (!ws || ws_bytes < Lw.total) return fail(ASR_E_WORKSPACE, "asr_conv_backward_k: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  unsigned char* base = (unsigned char*)ws;
  float* dz = (float*)(base + Lw.dz);
  float* slabs = (float*)(base + Lw.slabs);
  const bool euler = mode == ASR_MODE_EULER;
  ASR_TRY(make_dz(euler ? F_EULER : F_CONV, dy, mask, nullptr, h, N, H, W, C, 0, dz, s));
  if (dx) ASR_TRY(conv_f32_k(euler ? B_EULER : B_CONV, kernel_size, dz, dx, nullptr, w, nullptr, h, 2.f * gamma, dy, N, H,
                             W, C, s, nullptr));
  if (dtheta || dbias || dw) {
    int nsl = 0;
    ASR_TRY(wgrad_f32(x, 0, dz, N, H, W, C, C, slabs, &nsl, s, kernel_size));
    ASR_TRY(reduce_and_project(slabs, nsl, (long)kernel_size * kernel_size * C * C, C, dtheta ? theta_dst : nullptr,
                               n_theta, dtheta, dbias, dw, (float*)(base + Lw.red), s));
  }
  return ASR_OK;
}

size_t asr_conv_backward_workspace_bytes(int N, int H, int W, int C, int dtype) {
  if (check_shape(N, H, W, C) != ASR_OK) return 0;
  return bwd_ws_layout(N, H, W, C, dtype).total;
}

int asr_conv_backward(int mode, const void* dy, const void* x, const uint8_t* mask, const void* w,
                      const int32_t* theta_dst, long n_theta, float h, float gamma, int N, int H, int W, int C,
                      int dtype, void* dx, float* dtheta, float* dbias, float* dw_hwio, void* ws, size_t ws_bytes,
                      asr_stream_t stream) {
  ASR_TRY(check_shape(N, H, W, C));
  if (mode != ASR_MODE_EULER && mode != ASR_MODE_CONV) return fail(ASR_E_ARG, "asr_conv_backward: bad mode %d", mode);
  if (!dy || !w || (mode == ASR_MODE_EULER && !mask)) return fail(ASR_E_ARG, "asr_conv_backward: null pointer");
  if ((dtheta || dbias || dw_hwio) && !x) return fail(ASR_E_ARG, "asr_conv_backward: x needed for weight gradients");
  if (dtheta && !theta_dst) return fail(ASR_E_ARG, "asr_conv_backward: theta_dst needed for dtheta");
  if (dtype != ASR_F32 && dtype != ASR_BF16) return fail(ASR_E_ARG, "asr_conv_backward: bad dtype");
  if (dtype == ASR_BF16 && !mfma_supported(C, W) && !convb_supported(W, C))
    return fail(ASR_E_UNSUPPORTED, "bf16 conv needs C in {16,32,64} and W in {32, 16, 8} (C=%d W=%d)",
                C, W);
  if (!ws || ws_bytes < bwd_ws_layout(N, H, W, C, dtype).total)
    return fail(ASR_E_WORKSPACE, "asr_conv_backward: workspace too small");
  return conv_backward_impl(mode, dy, x, mask, w, theta_dst, n_theta, h, gamma, N, H, W, C, dtype, dx, dtheta, dbias,
                            dw_hwio, ws, (hipStream_t)stream);
}

static int check_block_args(const char* fn, int N, int H, int W, int C, int dtype) {
  ASR_TRY(check_shape(N, H, W, C));
  if (dtype != ASR_F32 && dtype != ASR_BF16) return fail(ASR_E_ARG, "%s: bad dtype %d", fn, dtype);
  if (dtype == ASR_BF16 && !mfma_supported(C, W))
    return fail(ASR_E_UNSUPPORTED, "%s: bf16 needs C in {16,32,64} and W == 32 (C=%d W=%d)", fn, C, W);
  return ASR_OK;
}

int asr_rk2_forward(const void* x, void* xmid, void* y, uint8_t* mask1, uint8_t* mask2, const void* w,
                    const float* bias, float h, int N, int H, int W, int C, int dtype, asr_stream_t stream) {
  ASR_TRY(check_block_args("asr_rk2_forward", N, H, W, C, dtype));
  if (!x || !xmid || !y || !w) return fail(ASR_E_ARG, "asr_rk2_forward: null pointer");
  if (x == xmid || x == y || xmid == y) return fail(ASR_E_ARG, "asr_rk2_forward: x, xmid and y must not alias");
  return rk2_forward_impl(x, xmid, y, mask1, mask2, w, bias, h, N, H, W, C, dtype, (hipStream_t)stream);
}

size_t asr_rk2_backward_workspace_bytes(int N, int H, int W, int C, int dtype) {
  if (check_shape(N, H, W, C) != ASR_OK) return 0;
  return bwd_ws_layout(N, H, W, C, dtype, 2).total;
}

int asr_rk2_backward(const void* dy, const void* x, const void* xmid, const uint8_t* mask1, const uint8_t* mask2,
                     const void* w, const int32_t* theta_dst, long n_theta, float h, float gamma, int N, int H, int W,
                     int C, int dtype, void* dx, float* dtheta, float* dbias, float* dw_hwio, void* ws,
                     size_t ws_bytes, asr_stream_t stream) {
  ASR_TRY(check_block_args("asr_rk2_backward", N, H, W, C, dtype));
  if (!dy || !x || !xmid || !mask1 || !mask2 || !w) return fail(ASR_E_ARG, "asr_rk2_backward: null pointer");
  if (dtheta && !theta_dst) return fail(ASR_E_ARG, "asr_rk2_backward: theta_dst needed for dtheta");
  const BwdWs L = bwd_ws_layout(N, H, W, C, dtype, 2);
  if (!ws || ws_bytes < L.total) return fail(ASR_E_WORKSPACE, "asr_rk2_backward: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  unsigned char* base = (unsigned char*)ws;
  float* slabs = (float*)(base + L.slabs);
  const bool need_w = dtheta || dbias || dw_hwio;
  int nsl = 0;
  ASR_TRY(rk2_backward_slabs(dy, x, xmid, mask1, mask2, w, h, gamma, N, H, W, C, dtype, dx, base + L.g, need_w, slabs,
                             (float*)(base + L.dz), &nsl, s));
  if (need_w)
    ASR_TRY(reduce_and_project(slabs, nsl, 9L * C * C, C, dtheta ? theta_dst : nullptr, n_theta, dtheta, dbias,
                               dw_hwio, (float*)(base + L.red), s));
  return ASR_OK;
}

long asr_net_param_count(const asr_net_config* cfg) {
  if (net_check(cfg) != ASR_OK) return -1;
  return net_layout(cfg).nparams;
}

size_t asr_net_workspace_bytes(const asr_net_config* cfg) {
  if (net_check(cfg) != ASR_OK) return 0;
  return net_layout(cfg).total;
}

int asr_net_prepare(const asr_net_config* cfg, void* ws, size_t ws_bytes) {
  ASR_TRY(net_check(cfg));
  const NetLayout L = net_layout(cfg);
  if (!ws || ws_bytes < L.total) return fail(ASR_E_WORKSPACE, "asr_net_prepare: workspace too small");
  ASR_TRY(check_ws_device(ws, "asr_net_prepare"));
  std::vector<int32_t> w_src((size_t)L.E), theta_dst((size_t)L.ntheta * 2);
  ASR_TRY(param_map(cfg->C, cfg->param_kind, cfg->antisymmetric, w_src.data(), theta_dst.data()));
  unsigned char* b = (unsigned char*)ws;
  if (L.sep_bwd && !L.inference) {
    std::vector<int32_t> w_bwd((size_t)L.E);
    ASR_TRY(param_map_transpose(cfg->C, w_src.data(), w_bwd.data()));
    ASR_TRY(hip_check(hipMemcpy(b + L.w_src_bwd, w_bwd.data(), w_bwd.size() * 4, hipMemcpyHostToDevice), "hipMemcpy"));
  }
  ASR_TRY(hip_check(hipMemcpy(b + L.w_src, w_src.data(), w_src.size() * 4, hipMemcpyHostToDevice), "hipMemcpy"));
  ASR_TRY(hip_check(hipMemcpy(b + L.theta_dst, theta_dst.data(), theta_dst.size() * 4, hipMemcpyHostToDevice),
                    "hipMemcpy"));
  if (L.stack_pair) {  // the same pull-back from k_bwd3_stack's pair-local D slabs
    std::vector<int32_t> pr(theta_dst.size());
    ASR_TRY(theta_dst_pair_host(theta_dst.data(), L.ntheta, cfg->C, pr.data()));
    ASR_TRY(hip_check(hipMemcpy(b + L.theta_dst_pr, pr.data(), pr.size() * 4, hipMemcpyHostToDevice), "hipMemcpy"));
  }
  if (L.stack_bwd) {  // the same map into k_bwd3_stack's tile-major dW slabs (ASR_VARIANT_FULL_SLABS)
    const int C = cfg->C;
    std::vector<int32_t> tm(theta_dst);
    for (auto& v : tm) {
      if (v < 0) continue;
      const long e = v >> 1, m = e / C, o = e % C;
      const long et = (((m / 16) * (C / 16) + o / 16) * 64 + 16 * ((m % 16) / 4) + o % 16) * 4 + m % 4;
      v = (int32_t)((et << 1) | (v & 1));
    }
    ASR_TRY(hip_check(hipMemcpy(b + L.theta_dst_tm, tm.data(), tm.size() * 4, hipMemcpyHostToDevice), "hipMemcpy"));
  }
  return ASR_OK;
}

int asr_net_forward(const asr_net_config* cfg, const float* params, const void* images, float* probs, void* ws,
                    size_t ws_bytes, asr_stream_t stream) {
  ASR_TRY(net_check(cfg));
  const NetLayout L = net_layout(cfg);
  if (!params || !images || !probs) return fail(ASR_E_ARG, "asr_net_forward: null pointer");
  if (!ws || ws_bytes < L.total) return fail(ASR_E_WORKSPACE, "asr_net_forward: workspace too small");
  ASR_TRY(check_ws_device(ws, "asr_net_forward"));
  hipStream_t s = (hipStream_t)stream;
  unsigned char* b = (unsigned char*)ws;
  unsigned char* xL = nullptr;
  ASR_TRY(net_forward_impl(cfg, L, params, images, false, b, s, &xL));
  ASR_TRY(head(xL, cfg->dtype == ASR_BF16, params + L.off_fck, params + L.off_fcb, nullptr, cfg->N, cfg->H * cfg->W,
               cfg->C, cfg->num_classes, probs, nullptr, nullptr, nullptr, nullptr, s));
  return ASR_OK;
}

int asr_net_check_status(const asr_net_config* cfg, const void* ws, size_t ws_bytes, asr_stream_t stream) {
  ASR_TRY(net_check(cfg));
  const NetLayout L = net_layout(cfg);
  if (!ws || ws_bytes < L.total) return fail(ASR_E_WORKSPACE, "asr_net_check_status: workspace too small");
  ASR_TRY(check_ws_device(ws, "asr_net_check_status"));
  // the stream's own completion status only (hipGetLastError would report, and clear,
  // whatever error another HIP call on this thread left behind)
  return hip_check(hipStreamSynchronize((hipStream_t)stream), "hipStreamSynchronize");
}

int asr_net_kernel_times(float* us) {
  if (!us) return fail(ASR_E_ARG, "asr_net_kernel_times: null output");
  const TimedEvents* t = timed_events_here();
  if (!t || !t->made || !(t->rec & 3u))
    return fail(ASR_E_ARG, "asr_net_kernel_times: no ASR_VARIANT_TIMED call recorded on the current device");
  for (int i = 0; i < 3; ++i) us[i] = -1.f;
  for (int i = 0; i < 3; ++i) {
    const int a = i == 0 ? 0 : i + 1, e = a + 1;
    if ((t->rec >> a & 1u) && (t->rec >> e & 1u)) {
      ASR_TRY(hip_check(hipEventSynchronize(t->ev[e]), "hipEventSynchronize"));
      float ms = 0.f;
      ASR_TRY(hip_check(hipEventElapsedTime(&ms, t->ev[a], t->ev[e]), "hipEventElapsedTime"));
      us[i] = ms * 1e3f;
    }
  }
  return ASR_OK;
}

int asr_net_forward_backward(const asr_net_config* cfg, const float* params, const void* images, const float* targets,
                             float* grads, float* loss, float* probs, void* ws, size_t ws_bytes,
                             asr_stream_t stream) {
  ASR_TRY(net_check(cfg));
  const NetLayout L = net_layout(cfg);
  if (!params || !images || !targets || !grads || !loss) return fail(ASR_E_ARG, "asr_net_forward_backward: null");
  if (!ws || ws_bytes < L.total) return fail(ASR_E_WORKSPACE, "asr_net_forward_backward: workspace too small");
  // before any launch: an inference layout has no backward buffers (its maps for the
  // transposed operator and the training activations are absent)
  if (L.inference)
    return fail(ASR_E_ARG, "asr_net_forward_backward: an ASR_VARIANT_INFERENCE workspace has no training buffers");
  ASR_TRY(check_ws_device(ws, "asr_net_forward_backward"));
  hipStream_t s = (hipStream_t)stream;
  unsigned char* b = (unsigned char*)ws;
  const int C = cfg->C, N = cfg->N, H = cfg->H, W = cfg->W, K = cfg->num_classes;
  const bool bf = cfg->dtype == ASR_BF16;
  const bool stacked = L.stack_bwd && !(cfg->variant & ASR_VARIANT_PER_BLOCK_BWD);
  ASR_TRY(net_forward_impl(cfg, L, params, images, true, b, s));
  auto act = [&](int i) { return b + L.acts + (size_t)i * L.P * L.act_bytes; };
  // head: probabilities, per-image loss, dlogits, dL/dx_L
  unsigned char* dcur = b + L.dxa;
  unsigned char* dnext = b + L.dxb;
  float* probs_ws = probs ? probs : (float*)(b + L.probs);
  // the stacked Euler backward stages its top block's dy from one row per image (the GAP gradient is
  // constant over the pixels): the head writes N x C values instead of the full dL/dx_L tensor
  const bool grow = stacked && !L.rk2 && !(cfg->variant & ASR_VARIANT_FULL_DXL);
  ASR_TRY(head(act(cfg->L), bf, params + L.off_fck, params + L.off_fcb, targets, N, H * W, C, K, probs_ws,
               (float*)(b + L.loss_per), (float*)(b + L.dlogits), (float*)(b + L.gap), grow ? nullptr : dcur, s,
               grow ? b + L.grow : nullptr));
  ASR_TRY(head_param_grads((const float*)(b + L.gap), (const float*)(b + L.dlogits), N, C, K, grads + L.off_fck,
                           grads + L.off_fcb, (const float*)(b + L.loss_per), loss, s));
  // blocks, last to first
  const int32_t* theta_dst = (const int32_t*)(b + L.theta_dst);
  int nsl_blk = 0;
  const BwdWs bw = bwd_ws_layout(N, H, W, C, cfg->dtype, L.stages, 3, bf ? -1 : 0);  // (net_layout's)
  int dz1_fused = 0;  // dcur holds dz1 = dx1 * [x1 > 0] after the block loop
  const float* pend_slabs = nullptr;  // the slabs whose pass-1 reduction is still pending
  int pend_P = 0;
  float* pend_grp = nullptr;
  const bool fold_on = !(cfg->variant & ASR_VARIANT_NO_FOLD);               // else the reduction as separate launches
  const bool stem_v1 = (cfg->variant & ASR_VARIANT_STEM_WGRAD_VALU) != 0;  // fp32 VALU stem wgrad
  ASR_TRY(timed_event(cfg, 2, s));  // (measurement) the blocks' backward starts
  if (L.deep) {  // C=16: all L blocks in one launch (dx resident in LDS), one slab set per layer
    int rows = 0, in_b = 0;
    float* slabs = (float*)(b + L.deep_slabs);
    ASR_TRY(deep16_backward(dcur, dnext, act(0), L.P, (const uint8_t*)(b + L.masks), L.mask_bytes,
                            b + (L.sep_bwd ? L.wbuf_bwd : L.wbuf), cfg->h, L.sep_bwd ? 0.f : 2.f * cfg->gamma, N,
                            cfg->L, slabs, &rows, &in_b, s));
    ASR_TRY(timed_event(cfg, 3, s));
    if (in_b) std::swap(dcur, dnext);
    const int G = reduce_groups(rows);
    ASR_TRY(reduce_slabs_to_groups(slabs, cfg->L * rows, L.E + C, (float*)(b + L.grp), s));
    ASR_TRY(project_layers((float*)(b + L.grp), (long)G * (L.E + C), G, L.E, C, theta_dst, L.ntheta, cfg->L,
                           grads + L.off_blk, L.blk_stride, s));
    ASR_TRY(timed_event(cfg, 4, s));
  }
  if (stacked) {  // C=64: all L blocks in one launch, tile-major slabs
    const int grid = L.stack_grid;
    const bool pair = L.stack_pair && !(cfg->variant & ASR_VARIANT_FULL_SLABS);
    const long ES = stack_slab_floats(C, pair ? 1 : 0), sst = (long)grid * ES;
    float* slabs = (float*)(b + L.stack_slabs);
    float* grp = (float*)(b + L.grp);
    // (RK2: the first block's first stage has the extra term, so the stem's relu' runs separately)
    const int ro0 = L.fast_stem && !stem_v1 && !L.rk2;
    int lfold = cfg->L;
    const uint8_t* m1 = (const uint8_t*)(b + L.masks);
    ASR_TRY(block_stack_bwd_mfma(dcur, dnext, act(0), L.P, m1, L.mask_bytes, b + (L.sep_bwd ? L.wbuf_bwd : L.wbuf),
                                 L.wstride, cfg->h, L.sep_bwd ? 0.f : 2.f * cfg->gamma, N, H, W, C, cfg->L, ro0, slabs,
                                 sst, grp, L.grp_stride, (unsigned*)(b + L.stack_done), &lfold, s,
                                 L.rk2 ? b + L.xmids : nullptr, L.rk2 ? m1 + (size_t)cfg->L * L.mask_bytes : nullptr,
                                 L.rk2 ? b + L.dxg : nullptr, grow ? b + L.grow : nullptr, fold_on ? 1 : 0,
                                 pair ? 1 : 0));
    ASR_TRY(timed_event(cfg, 3, s));
    // pass 1 of the blocks below lfold, and of any block whose in-launch fold was
    // flagged (a workgroup's wait ran out), before the projection reads them
    ASR_TRY(stack_bwd_reduce_rest(slabs, sst, grid, ES, grp, L.grp_stride, cfg->L, lfold,
                                  (const unsigned*)(b + L.stack_done), s));
    if (cfg->L & 1) std::swap(dcur, dnext);
    dz1_fused = ro0;
    ASR_TRY(project_layers(grp, L.grp_stride, reduce_groups(grid), ES - C, C,
                           (const int32_t*)(b + (pair ? L.theta_dst_pr : L.theta_dst_tm)), L.ntheta, cfg->L,
                           grads + L.off_blk, L.blk_stride, s));
    ASR_TRY(timed_event(cfg, 4, s));
  }
  for (int l = (L.deep || stacked) ? -1 : cfg->L - 1; l >= 0; --l) {
    const unsigned char* wl = b + (L.sep_bwd ? L.wbuf_bwd : L.wbuf) + (size_t)l * L.wstride * L.act_bytes;
    const uint8_t* mask = (const uint8_t*)(b + L.masks) + (size_t)l * L.mask_bytes;
    const float gam = L.sep_bwd ? 0.f : cfg->gamma;
    float* grp_l = (float*)(b + L.grp) + (size_t)l * L.grp_stride;
    // a block's slabs alternate between two buffers; pass 1 of the previous
    // (deeper) block's reduction rides in this block's (second-stage) kernel
    // when it can (else it runs here), and this block's waits for the next
    // block (or the end of the loop)
    // (fp32: every block keeps its own slabs; one launch reduces them all after the loop)
    float* slabs_l = !bf ? (float*)(b + L.slabs_all) + (size_t)l * L.slab_stride
                         : (float*)(b + ((l & 1) ? L.slabs2 : L.bwdws + bw.slabs));
    int nsl = 0, folded = 0;
    if (L.rk2) {
      const unsigned char* xm = b + L.xmids + (size_t)l * L.P * L.act_bytes;
      ASR_TRY(rk2_backward_slabs(dcur, act(l), xm, mask, mask + (size_t)cfg->L * L.mask_bytes, wl, cfg->h, gam, N, H,
                                 W, C, cfg->dtype, dnext, b + L.dxg, true, slabs_l, (float*)(b + L.bwdws + bw.dz),
                                 &nsl, s, fold_on ? pend_slabs : nullptr, fold_on ? pend_P : 0, pend_grp, &folded));
    } else {
      ASR_TRY(block_backward(ASR_MODE_EULER, dcur, act(l), mask, wl, cfg->h, gam, N, H, W, C, cfg->dtype, dnext, true,
                             nullptr, false, slabs_l, (float*)(b + L.bwdws + bw.dz), &nsl, s,
                             l == 0 && L.fast_stem && bf && !stem_v1, l == 0 ? &dz1_fused : nullptr,
                             fold_on ? pend_slabs : nullptr, fold_on ? pend_P : 0, pend_grp, &folded));
    }
    nsl_blk = nsl;
    std::swap(dcur, dnext);
    if (!bf) {
      if (nsl > L.stages * L.f32_rows)  // (the device differs from the one the workspace was sized on)
        return fail(ASR_E_WORKSPACE, "fp32 block %d wrote %d slab rows, the workspace holds %d (sized on another device?)",
                    l, nsl, L.stages * L.f32_rows);
      continue;
    }
    if (pend_P > 0 && !folded) ASR_TRY(reduce_slabs_to_groups(pend_slabs, pend_P, L.E + C, pend_grp, s));
    pend_slabs = slabs_l;
    pend_P = nsl;
    pend_grp = grp_l;
  }
  if (pend_P > 0) ASR_TRY(reduce_slabs_to_groups(pend_slabs, pend_P, L.E + C, pend_grp, s));
  if (!bf && !L.deep && !stacked && nsl_blk > 0)  // (every block of a network has the same slab count)
    ASR_TRY(reduce_slab_layers((const float*)(b + L.slabs_all), L.slab_stride, nsl_blk, L.E + C,
                               (float*)(b + L.grp), L.grp_stride, cfg->L, s));
  // pass 2 of every block's weight-gradient reduction + projection onto theta, one launch
  if (!L.deep && !stacked) {
    ASR_TRY(timed_event(cfg, 3, s));  // (per-block kernels: their slab passes ride inside)
    ASR_TRY(project_layers((float*)(b + L.grp), L.grp_stride, reduce_groups(nsl_blk), L.E, C, theta_dst, L.ntheta,
                           cfg->L, grads + L.off_blk, L.blk_stride, s));
    ASR_TRY(timed_event(cfg, 4, s));
  }
  // stem: dz1 = dx1 * [x1 > 0]; conv1 weight/bias gradient from the normalised input
  const long E1 = 9L * cfg->Cin * C;
  unsigned char* sw = b + L.bwdws;
  float* dz = (float*)sw;
  float* slabs = (float*)(sw + align_up((size_t)L.P * 4, 256));
  float* red = (float*)(sw + align_up((size_t)L.P * 4, 256) + align_up((size_t)kMaxSlabsApi * (E1 + C) * 4, 256));
  int nsl = 0;
  const float inv_std = cfg->use_norm ? 1.f / cfg->divide_by_stddev : 1.f;
  if (L.fast_stem && bf && !dz1_fused && !stem_v1 && stem_wgrad_mfma_supported(cfg->Cin, H, W, C) && L.P % 8 == 0) {
    const long n8 = (long)L.P / 8;
    hipLaunchKernelGGL(k_relu_grad_bf16, dim3((unsigned)std::min<long>((n8 + 255) / 256, 4096)), dim3(256), 0, s,
                       (bf16*)dcur, (const bf16*)act(0), n8);
    ASR_LAUNCH_CHECK("k_relu_grad_bf16");
    dz1_fused = 1;
  }
  if (L.fast_stem && dz1_fused && stem_wgrad_mfma_supported(cfg->Cin, H, W, C)) {
    ASR_TRY(stem_wgrad_mfma(images, cfg->input_u8, dcur, N, H, W, cfg->Cin, C, cfg->subtract_mean, inv_std,
                            cfg->use_norm, slabs, &nsl, s));
  } else if (L.fast_stem) {  // (masking an already-masked dz1 again is exact)
    ASR_TRY(stem_wgrad(images, cfg->input_u8, dcur, act(0), bf, N, H, W, cfg->Cin, C, cfg->subtract_mean, inv_std,
                       cfg->use_norm, slabs, &nsl, s));
  } else {
    ASR_TRY(make_dz(F_RELU, dcur, nullptr, act(0), 1.f, N, H, W, C, bf ? 1 : 0, dz, s));
    ASR_TRY(wgrad_f32(b + L.x0, 0, dz, N, H, W, cfg->Cin, C, slabs, &nsl, s));
  }
  ASR_TRY(reduce_and_project(slabs, nsl, E1, C, nullptr, 0, nullptr, grads + L.off_c1b, grads + L.off_c1k, red, s));
  return ASR_OK;
}

int asr_segment_sq_norms(const float* x, const long* offsets, int n_segments, float* out, asr_stream_t stream) {
  if (!x || !offsets || !out || n_segments < 0) return fail(ASR_E_ARG, "asr_segment_sq_norms: bad arguments");
  if (n_segments == 0) return ASR_OK;
  hipLaunchKernelGGL(k_segment_sq_norms, dim3(n_segments), dim3(256), 0, (hipStream_t)stream, x, offsets, out);
  ASR_LAUNCH_CHECK("k_segment_sq_norms");
  return ASR_OK;
}

int asr_batch_metrics(const float* probs, const float* targets, const float* loss, int N, int K, float* accum,
                      asr_stream_t stream) {
  if (!probs || !targets || !accum || N < 1 || K < 1) return fail(ASR_E_ARG, "asr_batch_metrics: bad args");
  hipLaunchKernelGGL(k_batch_metrics, dim3(1), dim3(256), 0, (hipStream_t)stream, probs, targets, loss, N, K, accum);
  ASR_LAUNCH_CHECK("k_batch_metrics");
  return ASR_OK;
}

int asr_adam_update(float* params, const float* grads, float* m, float* v, long n, float lr, float beta1, float beta2,
                    float eps, long step, float grad_scale, asr_stream_t stream) {
  if (!params || !grads || !m || !v || n < 0 || step < 1) return fail(ASR_E_ARG, "asr_adam_update: bad arguments");
  const double lr_t = (double)lr * sqrt(1.0 - pow((double)beta2, (double)step)) / (1.0 - pow((double)beta1, (double)step));
  const unsigned grid = (unsigned)std::max<long>(1, std::min<long>((n + 255) / 256, 4096));
  hipLaunchKernelGGL(k_adam, dim3(grid), dim3(256), 0, (hipStream_t)stream, params, grads, m, v, n, (float)lr_t,
                     beta1, beta2, eps, grad_scale);
  ASR_LAUNCH_CHECK("k_adam");
  return ASR_OK;
}

}  // extern "C"
