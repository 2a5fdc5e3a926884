/*
 * asr.h — C ABI of libasr.so, the MI355X-native hot path of the
 * antisymmetric-ResNet (pierluigiferrari/differential_equations_resnet).
 *
 * One Euler block of the reference is
 *     x_{n+1} = x_n + h * relu(conv3x3(x_n, W(theta)) + b)
 * (models/tfkeras_resnets.py:69-92) where W(theta) is re-materialised from the
 * layer's free parameters on every step
 * (layers/tfkeras_layer_Conv2DAntisymmetric3By3.py:85-171).
 *
 * Conventions
 *   - plain pointers and sizes only; every pointer is a device pointer unless
 *     the comment says "host";
 *   - activations NHWC, kernels HWIO [3][3][C_in][C_out] (reference layout);
 *   - every call is a stateless launch on the caller's stream; nothing here
 *     allocates device memory: workspaces are caller-owned, sized by the
 *     *_workspace_bytes queries;
 *   - every entry point returns 0 on success and a negative ASR_E* code on
 *     failure; asr_last_error() returns a thread-local message.  Nothing
 *     throws across the ABI.
 *
 * Each declaration cites the reference interface it replaces.
 */
#ifndef ASR_H_
#define ASR_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* asr_stream_t; /* a hipStream_t (0 = null stream) */

/* error codes */
#define ASR_OK 0
#define ASR_E_ARG (-1)         /* invalid argument (shape, dtype, null)       */
#define ASR_E_UNSUPPORTED (-2) /* valid but not implemented on this device    */
#define ASR_E_WORKSPACE (-3)   /* workspace too small                          */
#define ASR_E_HIP (-4)         /* HIP runtime error (see asr_last_error)       */
#define ASR_E_DEVICE (-5)      /* no usable gfx950 device                      */

/* activation dtypes */
#define ASR_F32 0
#define ASR_BF16 1

/* parametrisations of the antisymmetric kernel (what theta means) */
#define ASR_PARAM_3BY3 0    /* Conv2DAntisymmetric3By3: a,b,c,d then
                               input_kernels_for_output_kernel_{o}[3,3,C-o-1]
                               (…3By3.py:104-141, :219-245)                   */
#define ASR_PARAM_GENERAL 1 /* Conv2DAntisymmetric (kernel_size 3): per o the
                               centro_sym_{i}_{j} scalars then
                               input_kernels_for_output_kernel_{o}[3,3,C-o-1,1]
                               (…Conv2DAntisymmetric.py:109-145)              */
#define ASR_PARAM_REGULAR 2 /* plain Conv2D kernel [3,3,C,C] (the regular
                               identity block, tfkeras_resnets.py:76-83):
                               theta IS W in HWIO order                       */

/* block integrators (asr_net_config.integrator) */
#define ASR_INTEGRATOR_EULER 0
#define ASR_INTEGRATOR_RK2 1

/* conv modes */
#define ASR_MODE_EULER 0 /* y = x + h*relu(conv(x)+b); mask = [conv(x)+b > 0]
                            (tfkeras_resnets.py:69-92)                        */
#define ASR_MODE_CONV 1  /* y = conv(x) + b  (the layer's call(),
                            …3By3.py:157-171)                                 */

const char* asr_last_error(void);
int asr_abi_version(void);

/* Number of gfx950 compute units of the current device (0 on failure). */
int asr_device_cu_count(void);

/* ------------------------------------------------------------------------
 * Parametrisation (host-side, pure arithmetic)
 * --------------------------------------------------------------------- */

/* Number of free kernel parameters (no bias).  3BY3: 4C + 9C(C-1)/2.
 * Replaces the add_weight calls of …3By3.py:119-124, :219-245 and
 * …Conv2DAntisymmetric.py:123-128, :234-239. */
long asr_theta_count(int C, int kind, int antisymmetric);

/* Host: fill the element map of W(theta).
 *   w_src[e] for every HWIO element e = ((ky*3+kx)*C+i)*C+o:
 *      (j<<1)|neg  => W[e] = (neg ? -1 : +1) * theta[j]
 *      -1          => W[e] = gamma (non-trainable centre, …3By3.py:248-250)
 *   theta_dst[2*j+0], theta_dst[2*j+1]: the (<=2) W elements theta[j] feeds,
 *      encoded (e<<1)|neg, -1 if unused.  This is the pull-back used for the
 *      weight-gradient projection (autodiff of …3By3.py:115-141).
 * w_src: 9*C*C int32, theta_dst: 2*asr_theta_count int32 (host memory). */
int asr_param_map(int C, int kind, int antisymmetric, int32_t* w_src, int32_t* theta_dst);

/* Host: 1 if the operator A of this parametrisation satisfies
 * A + A^T = 2*gamma*I (3by3, general with antisymmetric=1), else 0; <0 on
 * bad arguments.  For such kinds the backward pass applies A^T with the
 * forward W (asr_conv_backward's identity).  Otherwise the caller
 * materialises the transposed operator W_bwd = -flip(W)^T from the map
 * asr_param_map_transpose returns and passes it (with gamma 0) as the
 * backward's w. */
int asr_param_is_antisymmetric(int kind, int antisymmetric);
int asr_param_map_transpose(int C, const int32_t* w_src, int32_t* w_src_bwd);
/* Host: the pull-back of an antisymmetric parametrisation (C = 64) from the
 * pair-local slabs of the stacked backward (asr_block_stack_backward, the
 * network's C=64 bf16 backward): every theta's entries (e, mirror(e)) of
 * theta_dst (asr_param_map) become 1 or 2 entries (s << 1 | neg) into a slab
 * of 74 16x16 tiles of D = dW - dW*^T (dW*[t][i][o] = dW[8-t][o][i]): tile
 * 16p + 4a + b holds D(tap p < 4, input tile a, output tile b); 64 + k the
 * tap-4 cross pair k; 70 + c tap 4's self tile c (raw, transposed for odd c);
 * element (r, c) of tile T at T*256 + ((r/4)*16 + c)*4 + r%4.  ASR_E_ARG when
 * some theta is not an antisymmetric pair. */
int asr_param_map_pair(int C, const int32_t* theta_dst, long n_theta, int32_t* theta_dst_pair);

/* Elements of the packed bf16 W consumed by the MFMA kernels. */
long asr_wpack_elems(int C);

/* Materialise W for L layers in one launch (replaces the per-step
 * slice/neg/concat/stack graph of …3By3.py:113-141).
 *   theta:  layer l's theta at theta + l*theta_stride (float32)
 *   w_src:  device copy of asr_param_map's w_src
 *   dtype == ASR_BF16: w_out (bf16) gets the MFMA fragment-packed layout,
 *                      layer l at l*w_stride elements.  Balanced rounding
 *                      (C <= 64, maps that pair every off-diagonal entry with
 *                      its antisymmetric partner: the 3by3 and general kinds):
 *                      each pair takes the bf16 neighbour that keeps every
 *                      output channel's sum of rounding errors near zero, so
 *                      W stays exactly antisymmetric and no channel carries a
 *                      fixed offset through a deep stack; otherwise round to
 *                      nearest.  Deterministic; restated bit-exactly by
 *                      tests/helpers.py w_bf16_balanced;
 *   dtype == ASR_F32:  w_out (float) gets plain HWIO [3][3][C][C]. */
int asr_theta_to_w(const float* theta, long theta_stride, int L, int C, const int32_t* w_src,
                   float gamma, void* w_out, long w_stride, int dtype, asr_stream_t stream);

/* ------------------------------------------------------------------------
 * Fused antisymmetric 3x3 conv / Euler block
 * --------------------------------------------------------------------- */

/* Forward.  mode ASR_MODE_EULER: y = x + h*relu(conv(x,W)+b), mask written;
 * ASR_MODE_CONV: y = conv(x,W)+b (mask may be NULL).
 *   x, y: [N,H,W,C] in dtype;  w: output of asr_theta_to_w for dtype;
 *   bias: C floats or NULL;  mask: asr_mask_bytes(N,H,W,C) bytes, relu bit of
 *   element (pixel, o) at bit index pixel*C + o (NHWC bit order, LSB first).
 * Replaces Conv2DAntisymmetric3By3.call (…3By3.py:157-171) and
 * single_layer_identity_block's relu/scale/add (tfkeras_resnets.py:89-92). */
int asr_conv_forward(int mode, const void* x, void* y, uint8_t* mask, const void* w,
                     const float* bias, float h, int N, int H, int W, int C, int dtype,
                     asr_stream_t stream);

long asr_mask_bytes(int N, int H, int W, int C);

/* Backward of asr_conv_forward (the autodiff of training.py:300 through the
 * block).  Given dy = dL/dy:
 *   EULER: dz = h*dy*mask;  dx = dy + A^T dz = dy - conv(dz,W) + 2*gamma*dz
 *   CONV:  dz = dy;         dx = A^T dz      =    - conv(dz,W) + 2*gamma*dz
 *   dW = sum_p patch(x) (x) dz, projected onto theta through theta_dst
 *   (device copy of asr_param_map's theta_dst); db = sum_p dz.
 * dtheta / dbias / dx may be NULL to skip that output; dw_hwio (float
 * [3][3][C][C], may be NULL) receives the unprojected dW.
 * ws: caller workspace of asr_conv_backward_workspace_bytes bytes. */
/* A stack of L Euler blocks in one call (the deep-stack path, BASELINE
 * config C3: single_layer_identity_block applied L times,
 * tfkeras_resnets.py:579-582).  Layer l reads x_l (x0 for l = 0) and writes
 * x_{l+1} to ys + l*y_stride elements and its relu mask to masks +
 * l*mask_stride bytes (masks may be NULL); with store_all == 0 only x_L is
 * written, to ys.  w: layer l's asr_theta_to_w output at w + l*w_stride
 * elements; bias: layer l's at bias + l*bias_stride (may be NULL).  bf16 at
 * C=16, H=W=32 runs all L steps in one launch with every image resident in
 * LDS; bf16 at C=64, W=32 (store_all) runs all L steps in one launch with
 * whole images per workgroup; other shapes run the per-block kernels in
 * sequence. */
int asr_block_stack_forward(const void* x0, void* ys, long y_stride, uint8_t* masks, long mask_stride,
                            const void* w, long w_stride, const float* bias, long bias_stride, float h,
                            int N, int H, int W, int C, int L, int dtype, int store_all, asr_stream_t stream);

/* Backward of asr_block_stack_forward over all L blocks: dyL = dL/dx_L;
 * xs: x_l at xs + l*x_stride elements (x_0 first, i.e. the stack's input
 * followed by its stored outputs); masks / w as the forward.  dx0 receives
 * dL/dx_0; dparams (may be NULL) layer l's [dtheta (n_theta) | dbias (C)] at
 * dparams + l*(n_theta + C), projected through theta_dst.  bf16 at C=16,
 * H=W=32 runs one fused launch with dx resident in LDS (w_stride must be
 * asr_wpack_elems(16)); bf16 at C=64, W=32 runs one launch over all blocks
 * (whole images per workgroup, weight-gradient slabs reduced in-launch);
 * other shapes run asr_conv_backward per block. */
size_t asr_block_stack_backward_workspace_bytes(int N, int H, int W, int C, int L, int dtype);
int asr_block_stack_backward(const void* dyL, const void* xs, long x_stride, const uint8_t* masks, long mask_stride,
                             const void* w, long w_stride, const int32_t* theta_dst, long n_theta, float h,
                             float gamma, int N, int H, int W, int C, int L, int dtype, void* dx0, float* dparams,
                             void* ws, size_t ws_bytes, asr_stream_t stream);

size_t asr_conv_backward_workspace_bytes(int N, int H, int W, int C, int dtype);
int asr_conv_backward(int mode, const void* dy, const void* x, const uint8_t* mask,
                      const void* w, const int32_t* theta_dst, long n_theta, float h,
                      float gamma, int N, int H, int W, int C, int dtype, void* dx,
                      float* dtheta, float* dbias, float* dw_hwio, void* ws, size_t ws_bytes,
                      asr_stream_t stream);

/* ------------------------------------------------------------------------
 * Conv2DAntisymmetric(kernel_size = k) for odd k != 3
 * (layers/tfkeras_layer_Conv2DAntisymmetric.py:60-68, 109-145, 163-170):
 * the same operator family on a k x k kernel (k = 3 is the functions above).
 * fp32 (the reference's precision); W HWIO [k,k,C,C]; maps of k*k*C*C
 * entries.  The antisymmetric kinds keep A^T = -A + 2 gamma I, so
 * asr_conv_backward_k takes the forward W (else W_bwd of
 * asr_param_map_transpose_k with gamma 0), as asr_conv_backward.
 * ---------------------------------------------------------------------- */
long asr_theta_count_k(int C, int kernel_size, int kind, int antisymmetric);
int asr_param_map_k(int C, int kernel_size, int kind, int antisymmetric, int32_t* w_src, int32_t* theta_dst);
int asr_param_map_transpose_k(int C, int kernel_size, const int32_t* w_src, int32_t* w_src_bwd);
int asr_theta_to_w_k(const float* theta, long theta_stride, int L, int C, int kernel_size, const int32_t* w_src,
                     float gamma, float* w_out, long w_stride, asr_stream_t stream);
int asr_conv_forward_k(int mode, int kernel_size, const float* x, float* y, uint8_t* mask, const float* w,
                       const float* bias, float h, int N, int H, int W, int C, asr_stream_t stream);
size_t asr_conv_backward_workspace_bytes_k(int N, int H, int W, int C, int kernel_size);
int asr_conv_backward_k(int mode, int kernel_size, const float* dy, const float* x, const uint8_t* mask,
                        const float* w, const int32_t* theta_dst, long n_theta, float h, float gamma, int N, int H,
                        int W, int C, float* dx, float* dtheta, float* dbias, float* dw, void* ws, size_t ws_bytes,
                        asr_stream_t stream);

/* ------------------------------------------------------------------------
 * RK2 (explicit midpoint) block — an EXTENSION, not in the reference
 * (BASELINE.json config 5; the reference integrates with forward Euler,
 * tfkeras_resnets.py:69-92).  Same W and bias in both stages:
 *   xmid = x + (h/2)*relu(conv(x,W)+b)      mask1 = [conv(x,W)+b > 0]
 *   y    = x + h*relu(conv(xmid,W)+b)       mask2 = [conv(xmid,W)+b > 0]
 * Each stage is the fused Euler kernel (the second takes its residual from x).
 * xmid and both masks are kept for the backward; masks may be NULL for
 * inference.
 * --------------------------------------------------------------------- */
int asr_rk2_forward(const void* x, void* xmid, void* y, uint8_t* mask1, uint8_t* mask2, const void* w,
                    const float* bias, float h, int N, int H, int W, int C, int dtype,
                    asr_stream_t stream);

/* Backward of asr_rk2_forward: dz2 = h*dy*mask2, g = A^T dz2,
 * dz1 = (h/2)*g*mask1, dx = dy + g + A^T dz1; dW = patch(x) (x) dz1 +
 * patch(xmid) (x) dz2 projected onto theta; db = sum(dz1 + dz2).
 * Outputs as asr_conv_backward; ws of asr_rk2_backward_workspace_bytes. */
size_t asr_rk2_backward_workspace_bytes(int N, int H, int W, int C, int dtype);
int asr_rk2_backward(const void* dy, const void* x, const void* xmid, const uint8_t* mask1,
                     const uint8_t* mask2, const void* w, const int32_t* theta_dst, long n_theta,
                     float h, float gamma, int N, int H, int W, int C, int dtype, void* dx,
                     float* dtheta, float* dbias, float* dw_hwio, void* ws, size_t ws_bytes,
                     asr_stream_t stream);

/* A stack of L RK2 blocks in one call (config 5's network path): block l reads
 * x_l (x0 for l = 0), writes x_mid_l to xmids + l*y_stride and x_{l+1} to
 * ys + l*y_stride elements, mask1 / mask2 of block l to masks1 / masks2 +
 * l*mask_stride bytes; w, bias as asr_block_stack_forward.  bf16 at C=64,
 * W=32 (>= 4 row bands per image) runs all 2L stages in one launch; other
 * shapes return ASR_E_UNSUPPORTED. */
int asr_rk2_stack_forward(const void* x0, void* ys, void* xmids, long y_stride, uint8_t* masks1, uint8_t* masks2,
                          long mask_stride, const void* w, long w_stride, const float* bias, long bias_stride, float h,
                          int N, int H, int W, int C, int L, int dtype, asr_stream_t stream);

/* Backward of asr_rk2_stack_forward: dyL = dL/dx_L; x_l at xs + l*x_stride
 * (x_0 first), x_mid_l at xmids + l*x_stride; dx0, dparams as
 * asr_block_stack_backward.  One launch over all blocks' two stages (bf16,
 * C=64, W=32). */
size_t asr_rk2_stack_backward_workspace_bytes(int N, int H, int W, int C, int L, int dtype);
int asr_rk2_stack_backward(const void* dyL, const void* xs, const void* xmids, long x_stride, const uint8_t* masks1,
                           const uint8_t* masks2, long mask_stride, const void* w, long w_stride,
                           const int32_t* theta_dst, long n_theta, float h, float gamma, int N, int H, int W, int C,
                           int L, int dtype, void* dx0, float* dparams, void* ws, size_t ws_bytes,
                           asr_stream_t stream);

/* ------------------------------------------------------------------------
 * Whole single-block network (get_single_block_resnet_build_function,
 * tfkeras_resnets.py:511-604, antisymmetric, num_stages=2, strides (1,1),
 * no BN/pooling):  normalise -> conv1+relu -> L Euler blocks -> GAP ->
 * Dense(num_classes, softmax); loss = mean Keras categorical cross-entropy
 * on the probabilities (training.py:295).
 * Parameters are ONE float32 buffer in Keras get_weights() order:
 *   conv1 kernel [3,3,Cin,C], conv1 bias [C],
 *   L x (theta [asr_theta_count(C, param_kind, antisymmetric)], bias [C]),
 *   fc kernel [C,K], fc bias [K].
 * --------------------------------------------------------------------- */
typedef struct asr_net_config {
  int N, H, W, Cin, C, L, num_classes;
  float h, gamma;
  float subtract_mean, divide_by_stddev; /* applied when use_norm != 0   */
  int use_norm;
  int dtype;    /* activation dtype: ASR_F32 or ASR_BF16                */
  int input_u8; /* images are uint8 (1) or float32 (0), NHWC            */
  int param_kind;    /* ASR_PARAM_3BY3 / _GENERAL / _REGULAR of the blocks */
  int antisymmetric; /* Conv2DAntisymmetric(antisymmetric=...); 1 otherwise */
  int integrator;    /* ASR_INTEGRATOR_EULER (the reference's block) or
                        ASR_INTEGRATOR_RK2 (extension, asr_rk2_forward)     */
  int variant;       /* 0 = the production kernel composition; ASR_VARIANT_*
                        bits select slower, independently written kernels
                        for the same math (cross-checks in the tests)      */
} asr_net_config;

/* asr_net_config.variant bits (all 0 in production) */
#define ASR_VARIANT_NO_FOLD 1      /* reduce every block's weight-gradient slabs in
                                      its own launch instead of folding the pass
                                      into the next block's backward kernel; the
                                      C=64 stacked backward then has no in-launch
                                      hand-off (a cross-check arm: without it a
                                      missed hand-off degrades gracefully)       */
#define ASR_VARIANT_STEM_FWD_VALU 2 /* bf16 stem forward on the fp32 VALU kernel  */
#define ASR_VARIANT_STEM_WGRAD_VALU 4 /* stem weight gradient on the fp32 VALU
                                        kernel from dx1 and x1 (relu' not fused
                                        into the first block's backward)       */
#define ASR_VARIANT_PER_BLOCK_FWD 8 /* C=64 bf16 training forward: one k_fwd3
                                       launch per block instead of the single
                                       all-blocks k_fwd3_stack launch         */
#define ASR_VARIANT_PER_BLOCK_BWD 16 /* C=64 bf16 Euler backward: one k_bwd3 launch
                                        per block (slab pass folded into the
                                        next one) instead of k_bwd3_stack     */
#define ASR_VARIANT_INFERENCE 32  /* forward-only workspace: x_0 and two ping-pong
                                     activation slots, no masks / backward
                                     buffers (asr_net_forward only; the C=64 bf16
                                     blocks run as one k_fwd3_stack launch)     */
#define ASR_VARIANT_TIMED 64      /* record HIP events around the block launches
                                     (measurement; asr_net_kernel_times)       */
#define ASR_VARIANT_FULL_DXL 128  /* C=64 bf16 Euler stacked backward: the head
                                     writes dL/dx_L as a full [N,H,W,C] tensor
                                     that the top block reads, instead of the
                                     per-image row it is constant over
                                     (cross-check of the synthesised dy)        */
#define ASR_VARIANT_FULL_SLABS 256 /* C=64 bf16 stacked backward of an antisymmetric
                                      operator: publish the full dW (144 tiles per
                                      workgroup slab) instead of the pair-local
                                      D = dW - dW*^T (74 tiles) the projection
                                      needs (cross-check and A/B arm)           */
#define ASR_VARIANT_W_BF16 512    /* bf16 networks: W rounded to nearest bf16
                                     instead of asr_theta_to_w's balanced
                                     rounding.  Same speed; the nearest
                                     rounding offsets every output channel by
                                     a fixed sum that every pixel of every
                                     layer sees, and over C3's 108 blocks that
                                     reaches 2.7e-2 relative L2 of a block's
                                     gradient vs the fp32 reference
                                     (tests/test_gpu_depth.py)    */

long asr_net_param_count(const asr_net_config* cfg);
size_t asr_net_workspace_bytes(const asr_net_config* cfg);
/* One-time setup of a workspace (uploads the parameter maps; blocking). */
int asr_net_prepare(const asr_net_config* cfg, void* ws, size_t ws_bytes);
/* probs: [N, K] float (softmax outputs, the Model's output). */
int asr_net_forward(const asr_net_config* cfg, const float* params, const void* images,
                    float* probs, void* ws, size_t ws_bytes, asr_stream_t stream);
/* One training forward+backward: targets [N,K] float (one-hot);
 * grads: same layout as params (overwritten); loss: 1 float (batch mean);
 * probs may be NULL. */
int asr_net_forward_backward(const asr_net_config* cfg, const float* params, const void* images,
                             const float* targets, float* grads, float* loss, float* probs,
                             void* ws, size_t ws_bytes, asr_stream_t stream);
/* Host, blocking (synchronises the stream): ASR_OK, or ASR_E_HIP with the
 * runtime's error when work on the stream failed (the stream's status only:
 * a pending error of another HIP call on this thread is neither reported nor
 * cleared).  (Since ABI 6 a missed
 * in-launch hand-off of the C=64 stacked backward is not an error: it costs
 * speed, see asr_stack_status.) */
int asr_net_check_status(const asr_net_config* cfg, const void* ws, size_t ws_bytes, asr_stream_t stream);

/* Host, blocking: device times in microseconds of the last asr_net_forward /
 * asr_net_forward_backward called with ASR_VARIANT_TIMED: us[0] the L blocks'
 * forward (the single stack launch where one runs), us[1] the L blocks'
 * backward kernels (the single stack launch k_bwd3_stack / k_bwd16_fused
 * where one runs), us[2] the weight-gradient reductions left after them and
 * the projection onto theta; -1 for a part that call did not run. */
int asr_net_kernel_times(float* us);

/* Host, blocking (a device-to-host copy on the current device): the number of
 * degraded in-launch slab hand-offs of the C=64 stacked backward (k_bwd3_stack)
 * since the last reset, >= 0 (or a negative error code).  A workgroup whose
 * bounded wait (~1-2 ms) for the other workgroups' weight-gradient slabs of a
 * block runs out flags that block and stops waiting for the rest of its
 * launch; the flagged blocks' slab reduction is then recomputed after the
 * launch, on the same stream, before the projection: the gradients are those
 * of the full hand-off, only slower (e.g. a grid that is not co-resident
 * because another kernel or process shares the device).  reset != 0 clears
 * the count in the same device atomic that reads it (a backward running on
 * another stream meanwhile loses no count). */
int asr_stack_status(int reset);
/* Test knob: force the stacked backward's grid (0: one workgroup per CU;
 * larger than the resident capacity makes hand-offs run out and degrade, see
 * asr_stack_status).  Workspace sizes depend on the grid: query them after
 * setting it. */
int asr_debug_stack_backward(int grid);

/* ------------------------------------------------------------------------
 * Multi-stage single-block ResNet (ABI 7): get_single_block_resnet_build_function
 * with num_stages > 2 (models/tfkeras_resnets.py:547-597), e.g. the He-style
 * ResNet-32: conv1 (3x3 'same', stride 1) + relu, then stages of identity Euler
 * blocks at 32^2 x 16, 16^2 x 32, 8^2 x 64; a stage whose filters or stride
 * change opens with single_layer_conv_block (tfkeras_resnets.py:204-269):
 *     y = relu(conv_3x3(x, K2, stride) + b2) + conv_1x1(x, K1, stride) + b1
 * (the 3x3 'same' with TF's asymmetric stride padding, the 1x1 'valid'), then
 * GAP + Dense softmax.  fp32 (the reference's precision); no BN / pooling.
 * ---------------------------------------------------------------------- */

/* The transition alone.  x [N,H,W,Ci] -> y [N,Ho,Wo,Co], Ho = ceil(H/stride);
 * k2 HWIO [3,3,Ci,Co], k1 [1,1,Ci,Co]; mask: N*Ho*Wo*Co bytes, 1 where
 * conv_3x3 + b2 > 0 (may be NULL).  Replaces single_layer_conv_block's
 * Conv2D '2' / '1' + relu + add (tfkeras_resnets.py:238-269). */
int asr_transition_forward(const float* x, float* y, uint8_t* mask, const float* k2, const float* b2,
                           const float* k1, const float* b1, int N, int H, int W, int Ci, int Co, int stride,
                           asr_stream_t stream);
/* Its backward: dx = dL/dx (may be NULL); dparams (may be NULL): the
 * gradients [dK2 | db2 | dK1 | db1] contiguous (the parameter order of
 * asr_stages_config). */
size_t asr_transition_backward_workspace_bytes(int N, int H, int W, int Ci, int Co, int stride);
int asr_transition_backward(const float* dy, const float* x, const uint8_t* mask, const float* k2, const float* k1,
                            int N, int H, int W, int Ci, int Co, int stride, float* dx, float* dparams, void* ws,
                            size_t ws_bytes, asr_stream_t stream);

#define ASR_STAGES_MAX 8
typedef struct asr_stages_config {
  int N, H, W, Cin, num_classes;
  int n_stages;               /* identity-block stages (the reference's num_stages - 1) */
  int C[ASR_STAGES_MAX];      /* filters of stage s (C[0] = conv1's filters)           */
  int L[ASR_STAGES_MAX];      /* identity blocks of stage s (>= 0)                     */
  int stride[ASR_STAGES_MAX]; /* s > 0: the opening transition's stride (1 or 2), 0 =
                                 no transition (then C[s] == C[s-1]); stride[0] = 0   */
  float h, gamma;
  float subtract_mean, divide_by_stddev; /* applied when use_norm != 0 */
  int use_norm, input_u8, param_kind, antisymmetric;
  int dtype;                  /* ABI 8: ASR_F32 (0) or ASR_BF16: the identity blocks'
                                 activations and convs (bf16 MFMA, fp32 accumulation
                                 and weight gradients); the transitions compute in fp32 */
} asr_stages_config;
/* params / grads (float32): conv1 kernel [3,3,Cin,C0], bias [C0]; per stage s:
 * the transition (if any) K2 [3,3,C[s-1],C[s]], b2, K1 [1,1,C[s-1],C[s]], b1,
 * then L[s] x (theta [asr_theta_count(C[s], param_kind, antisymmetric)], bias
 * [C[s]]); fc kernel [C_last, K], bias [K]. */
/* ASR_OK, or the code (and asr_last_error) the calls below fail with for this
 * config: ASR_E_ARG for a malformed one, ASR_E_UNSUPPORTED for a shape the
 * kernels do not take (e.g. a bf16 stage outside C {16,32,64} x W {32,16,8}).
 * ABI 8.  Host only. */
int asr_stages_check(const asr_stages_config* cfg);
long asr_stages_param_count(const asr_stages_config* cfg);
size_t asr_stages_workspace_bytes(const asr_stages_config* cfg);
int asr_stages_prepare(const asr_stages_config* cfg, void* ws, size_t ws_bytes);
int asr_stages_forward(const asr_stages_config* cfg, const float* params, const void* images, float* probs,
                       void* ws, size_t ws_bytes, asr_stream_t stream);
int asr_stages_forward_backward(const asr_stages_config* cfg, const float* params, const void* images,
                                const float* targets, float* grads, float* loss, float* probs, void* ws,
                                size_t ws_bytes, asr_stream_t stream);

/* tf.train.AdamOptimizer.apply_gradients (training.py:300-301), TF1
 * epsilon-hat form; step is the 1-based update count; g is multiplied by
 * grad_scale first (1/world for data-parallel mean). */
int asr_adam_update(float* params, const float* grads, float* m, float* v, long n, float lr,
                    float beta1, float beta2, float eps, long step, float grad_scale,
                    asr_stream_t stream);

/* ------------------------------------------------------------------------
 * Training-loop metrics, accumulated on the device (no per-step host sync).
 * ---------------------------------------------------------------------- */

/* out[i] = sum_{j in [offsets[i], offsets[i+1])} x[j]^2 for i < n_segments
 * (offsets: device int64 [n_segments+1]).  The per-layer gradient
 * mean-norm ||g|| / size of training.py:356-409 is sqrt(out[i]) / size. */
int asr_segment_sq_norms(const float* x, const long* offsets, int n_segments, float* out,
                         asr_stream_t stream);

/* Streaming mean loss + accuracy (tf.metrics.mean / tf.metrics.accuracy,
 * training.py:316-354): accum[0] += *loss, accum[1] += #{argmax probs ==
 * argmax targets}, accum[2] += N, accum[3] += 1.  loss may be NULL: the
 * batch-mean Keras categorical cross-entropy of probs is used (evaluation). */
int asr_batch_metrics(const float* probs, const float* targets, const float* loss, int N, int K,
                      float* accum, asr_stream_t stream);

/* ------------------------------------------------------------------------
 * Data-parallel collectives (RCCL over xGMI; one process per GPU).  NEW: the
 * reference is single-device (experiments_antisymmetric_resnet_v6.ipynb:361);
 * SURVEY.md §8(e) adds one all-reduce of the flat fp32 gradient buffer per
 * step (the batch is split by image: no BatchNorm, batch-mean loss,
 * training.py:295) and one broadcast of the initial parameters.
 * ---------------------------------------------------------------------- */
#define ASR_DIST_UNIQUE_ID_BYTES 128

/* Host: rank 0 creates the communicator id (out: 128 host bytes) and hands
 * it to every rank out of band (file, TCP store, ...). */
int asr_dist_unique_id(void* out);
/* Host, blocking, collective over all ranks: create this process's
 * communicator on the current HIP device. */
int asr_dist_init(int rank, int world, const void* unique_id);
/* In place on the caller's stream: buf = sum over ranks (dtype ASR_F32/BF16). */
int asr_dist_allreduce_sum(void* buf, size_t count, int dtype, asr_stream_t stream);
/* In place on the caller's stream: buf = root's buf. */
int asr_dist_broadcast(void* buf, size_t count, int dtype, int root, asr_stream_t stream);
/* World size of the live communicator (0 when none). */
int asr_dist_world_size(void);
/* Destroy the communicator (no-op without one). */
int asr_dist_finalize(void);

#ifdef __cplusplus
}
#endif
#endif /* ASR_H_ */
