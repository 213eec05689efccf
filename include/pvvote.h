/*
 * pvvote.h -- C ABI of libpvvote.so, the MI355X (gfx950) implementation of
 * PVNet's pixel-wise RANSAC keypoint voting.
 *
 * Reference interface being replaced (kennege/pvnet):
 *   lib/ransac_voting_gpu_layer/src/ransac_voting.cpp        (BND)  pybind11 module `ransac_voting`
 *   lib/ransac_voting_gpu_layer/src/ransac_voting_kernel.cu  (KU)   launchers + kernels
 *   lib/ransac_voting_gpu_layer/ransac_voting_gpu.py         (RV)   Python voting layers
 *
 * Conventions
 *   - Every pointer is a DEVICE pointer (hipMalloc / torch CUDA tensor memory)
 *     unless the comment says otherwise.  Sizes are element counts.
 *   - Every call is asynchronous on `stream` (a hipStream_t; NULL = the null
 *     stream) and performs no host synchronisation, so the calls can be
 *     captured into a hipGraph.  The pipelines allocate nothing (caller
 *     workspace); pv_voting_for_hypothesis needs no scratch at all (one
 *     kernel reads direct/coords/hypo and writes the mask).
 *   - Return value: 0 on success; a positive hipError_t from the launch; or a
 *     negative PV_E* code for a bad argument.  Nothing ever calls exit()
 *     (the reference's gpuAssert does, cuda_common.h:19-26).
 *   - Numerics: fp32 IEEE, no contraction, correctly rounded sqrt/div on every
 *     decision the reference makes; results are bit-identical to the
 *     reference arithmetic (see DESIGN.md "Exactness of the fast vote test").
 */
#ifndef PVVOTE_H_
#define PVVOTE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *pv_stream_t; /* hipStream_t */

#define PV_OK 0
#define PV_EINVAL (-1)     /* bad size / pointer / enum */
#define PV_EWORKSPACE (-2) /* workspace missing or too small */
#define PV_EALIGN (-3)     /* pointer not aligned as documented */

/* mask / segmentation encodings accepted by the pipelines */
#define PV_MASK_I64 0      /* int64 [b,H,W]; v3: (uint8)m != 0 (RV:533 .byte()); EVD: m == 1 (RV:340) */
#define PV_MASK_U8 1       /* uint8/bool [b,H,W]; same predicates on the byte value */
#define PV_MASK_I32 2      /* int32 [b,H,W] */
#define PV_MASK_SEG_F32 3  /* seg_pred logits f32 [b,2,H,W]: argmax(seg,1)==1 fused (DEMO:52) */
#define PV_MASK_SEG_F16 4  /* seg_pred logits f16 [b,2,H,W] */

#define PV_VERTEX_F32 0
#define PV_VERTEX_F16 1

#define PV_VOTE_OR 0       /* reference semantics: set 1 where inlier, leave other bytes (KU:124-125) */
#define PV_VOTE_DENSE 1    /* overwrite every byte with 0/1 (identical for the zero tensors every RV call site passes) */

const char *pv_version(void);
const char *pv_build_config(void); /* the build's compile-time kernel choices and grid shapes (static string) */
const char *pv_error_string(int code);
int pv_device_arch(char *buf, int len); /* writes the gcnArchName of the current device (host pointer) */

/* ---- streams for concurrent callers (not in the reference: its callers are DataParallel worker
 * threads, tools/parallel.py:183-200, each on its own device and torch's current stream) ----
 * pv_stream_create: a new non-blocking HIP stream of its own on the current device (priority as
 * hipStreamCreateWithPriority; 0 = default).  torch.cuda.Stream() hands out one of 32 pooled streams
 * per priority, round robin, so the 33rd "new" stream is the 1st again: callers that need streams no
 * one else launches on (one per in-flight lane or per launching thread) take them from here.
 * pv_stream_capture_id: the id of the stream capture `stream` belongs to, 0 when it is not capturing
 * (host pointer `id`); scratch owned by one captured graph is keyed by it. */
int pv_stream_create(int32_t priority, pv_stream_t *out);
int pv_stream_destroy(pv_stream_t stream);
int pv_stream_capture_id(pv_stream_t stream, uint64_t *id);

/* ---- drop-in kernels: the four functions of the `ransac_voting` module ---- */

/* replaces generate_hypothesis (BND:20-31 -> KU:51-86).
 * direct f32 [tn,vn,2], coords f32 [tn,2], idxs i32 [hn,vn,2] -> hypo f32 [hn,vn,2]
 * (every element written; degenerate pairs give (0,0) as the reference's zero-initialised output, KU:75). */
int pv_generate_hypothesis(const float *direct, const float *coords, const int32_t *idxs, float *hypo,
                           int32_t tn, int32_t vn, int32_t hn, pv_stream_t stream);

/* replaces voting_for_hypothesis (BND:41-55 -> KU:129-167).
 * hypo f32 [hn,vn,2]; inliers u8 [hn,vn,tn] caller-owned; mode PV_VOTE_OR or PV_VOTE_DENSE. */
int pv_voting_for_hypothesis(const float *direct, const float *coords, const float *hypo, uint8_t *inliers,
                             int32_t tn, int32_t vn, int32_t hn, float inlier_thresh, int32_t mode,
                             pv_stream_t stream);

/* replaces generate_hypothesis_vanishing_point (BND:64-75 -> KU:231-266); hypo f32 [hn,vn,3]. */
int pv_generate_hypothesis_vp(const float *direct, const float *coords, const int32_t *idxs, float *hypo,
                              int32_t tn, int32_t vn, int32_t hn, pv_stream_t stream);

/* replaces voting_for_hypothesis_vanishing_point (BND:85-99 -> KU:313-351); OR semantics. */
int pv_voting_for_hypothesis_vp(const float *direct, const float *coords, const float *hypo, uint8_t *inliers,
                                int32_t tn, int32_t vn, int32_t hn, float inlier_thresh, pv_stream_t stream);

/* mask-free form of  inl = zeros(hn,vn,tn); voting_for_hypothesis(...); torch.sum(inl, 2)
 * (RV:563-567): counts i32 [hn,vn] (overwritten). */
int pv_vote_counts(const float *direct, const float *coords, const float *hypo, int32_t *counts,
                   int32_t tn, int32_t vn, int32_t hn, float inlier_thresh, pv_stream_t stream);

/* ---- batched pipelines: the Python layers of RV, fully on device ---- */

typedef struct pv_image_desc {
    const void *mask;       /* see PV_MASK_*; for SEG_* this is seg_pred */
    int32_t mask_kind;
    int64_t mask_strides[4];/* elements: [b,h,w] (unused 4th) or, for SEG_*, [b,c,h,w] */
    const void *vertex;     /* [b,H,W,vn,2] view, any strides (e.g. vertex_pred.permute(0,2,3,1).view(...)) */
    int32_t vertex_kind;    /* PV_VERTEX_F32 / PV_VERTEX_F16 */
    int64_t vertex_strides[5];
    int32_t b, H, W, vn;
} pv_image_desc;

typedef struct pv_vote_params {
    int32_t round_hyp_num;  /* hypotheses per round (RV:520 round_hyp_num) */
    float inlier_thresh;    /* RV:520 inlier_thresh */
    float confidence;       /* only sets the diagnostic iteration count */
    int32_t max_iter;
    int32_t min_num;        /* fewer foreground pixels -> zeros (RV:537) */
    int32_t max_num;        /* more -> Bernoulli(max_num/fg) downsampling (RV:543-546) */
    uint64_t seed;          /* device RNG seed for idxs / downsampling (the reference uses torch's device RNG) */
    const int32_t *idxs;    /* optional [b, n_hyp, vn, 2] pixel pairs to use instead of the RNG (parity tests) */
    const uint8_t *keep;    /* optional [b, H, W] downsampling keep-mask instead of the RNG (parity tests) */
    /* EVD only */
    int32_t min_hyp_num;    /* RV:333 min_hyp_num (rounds = ceil(min_hyp_num / round_hyp_num)) */
    int32_t topk;           /* RV:263 topk (estimate_voting_distribution only) */
} pv_vote_params;

/* optional device outputs for tests/diagnostics (any may be NULL) */
typedef struct pv_v3_diag {
    float *hyp;             /* [b, hn, vn, 2] hypotheses */
    int32_t *counts;        /* [b, vn, hn] inlier counts */
    int32_t *win_idx;       /* [b, vn] */
    float *win_ratio;       /* [b, vn] */
    int32_t *tn;            /* [b] compacted foreground pixels (0 = skipped) */
    int32_t *iters;         /* [b] iterations the reference's loop would run (RV:578-582) */
    float *ata;             /* [b, vn, 2, 2] */
    float *atb;             /* [b, vn, 2] */
    void *ev_vote_begin;    /* hipEvent_t recorded on `stream` right before / after the fused */
    void *ev_vote_end;      /* vote+count kernel (per-kernel timing in bench.py)                */
    void *ev_compact_end;   /* hipEvent_t recorded right after the compaction (k_fg_count +
                             * k_compact, the call's first two kernels)                         */
} pv_v3_diag;

size_t pv_v3_workspace_size(int32_t b, int32_t H, int32_t W, int32_t vn, int32_t n_hyp);
/* Kernel launches one pv_ransac_voting_v3 call of this shape makes (the graph nodes it adds when
 * captured): compaction (2), hypotheses (0 when k_compact makes them), vote (1 per 2^31-pair chunk),
 * refine (1).  Build-internal (not in the reference API); 0 for an invalid shape. */
int pv_v3_kernel_launches(int32_t b, int32_t H, int32_t W, int32_t vn, int32_t n_hyp);

/* ransac_voting_layer_v3 (RV:520-604) for a whole batch; out f32 [b,vn,2]. */
int pv_ransac_voting_v3(const pv_image_desc *img, const pv_vote_params *prm, float *out,
                        void *workspace, size_t workspace_bytes, const pv_v3_diag *diag, pv_stream_t stream);

/* ransac_voting_layer_v5 (RV:769-864): v3 (use v5's defaults in prm: inlier_thresh 0.999, max_iter 20,
 * min_num 5, max_num 100) plus conf f32 [b,vn] = inlier ratio of each refined keypoint at conf_thresh
 * (0.999 in the reference, RV:856-858); 0 for skipped images. */
int pv_ransac_voting_v5(const pv_image_desc *img, const pv_vote_params *prm, float conf_thresh, float *out,
                        float *conf, void *workspace, size_t workspace_bytes, const pv_v3_diag *diag,
                        pv_stream_t stream);

/* ransac_motion_voting (RV:966-987): out f32 [b,vn,2] = mean over the foreground (mask.byte() != 0) of
 * vertex + (col, row); zeros for an empty foreground.  mask kinds I64/U8/I32. */
int pv_ransac_motion_voting(const pv_image_desc *img, float *out, pv_stream_t stream);

/* estimate_voting_distribution_with_mean (RV:333-406): mean f32 [b,vn,2] (device, input),
 * cov out f32 [b,vn,2,2].  (The reference returns `mean` unchanged.) */
int pv_estimate_voting_distribution_with_mean(const pv_image_desc *img, const pv_vote_params *prm,
                                              const float *mean, float *cov, void *workspace,
                                              size_t workspace_bytes, pv_stream_t stream);

/* The same with the diag's timing events (ev_compact_end, ev_vote_begin / ev_vote_end around the
 * vote/count kernel at n_hyp = rounds x round_hyp_num); its other fields are ignored.  Diagnostics
 * only (bench.py's U4 line); not part of the reference's interface. */
int pv_estimate_voting_distribution_with_mean_diag(const pv_image_desc *img, const pv_vote_params *prm,
                                                   const float *mean, float *cov, void *workspace,
                                                   size_t workspace_bytes, const pv_v3_diag *diag,
                                                   pv_stream_t stream);

/* estimate_voting_distribution (RV:263-331): mean out [b,vn,2], cov out [b,vn,2,2].
 * topk ties at the k-th ratio are taken lowest-hypothesis-index first. */
int pv_estimate_voting_distribution(const pv_image_desc *img, const pv_vote_params *prm, float *mean,
                                    float *cov, void *workspace, size_t workspace_bytes, pv_stream_t stream);

/* ---- uncertainty-weighted PnP (the consumer of the EVD covariances), batched ---- */

#define PV_PNP_WEIGHTS 0   /* wgt: f64 [pn,3] (wxx, wxy, wyy) per image, as uncertainty_pnp() takes them */
#define PV_PNP_COV 1       /* wgt: f32 [pn,2,2] covariances -> inv(sqrtm(C)), 0 if C00 < 1e-6 or NaN
                            * (lib/utils/evaluation_utils.py:168-178), then uncertainty_pnp() */
#define PV_PNP_COV_V2 2    /* wgt: f32 [pn,2,2] -> isotropic 1 / max eig(C), 0 if C00 < 1e-5
                            * (uncertainty_pnp_v2, extend_utils.py:116-166) */

typedef struct pv_pnp_batch {
    int32_t b, pn;          /* images; points per image (4 <= pn <= 64) */
    int32_t mode;           /* PV_PNP_* */
    const float *pts2d;     /* [b][pn][2] image points (the voted keypoints) */
    const void *wgt;        /* see PV_PNP_*; [b][pn][...] */
    const double *pts3d;    /* [pn][3] model points, image i at pts3d + i * pts3d_stride */
    const double *K;        /* [3][3] camera matrix, image i at K + i * K_stride */
    int64_t pts3d_stride;   /* elements; 0 = one set shared by the batch */
    int64_t K_stride;       /* elements; 0 = shared */
    const double *pts2d64;  /* optional f64 [b][pn][2]: used instead of pts2d when non-NULL (the
                             * reference's cffi path hands float64 points to Ceres, extend_utils.py:80) */
} pv_pnp_batch;

/* optional device outputs (any may be NULL) */
typedef struct pv_pnp_diag {
    double *init_rt;        /* [b][6] the P3P initial pose (rvec, t) */
    int32_t *p3p_ok;        /* [b] 1 if P3P found a solution (cv2.solvePnP's return value) */
    int32_t *iterations;    /* [b] trust-region iterations */
    int32_t *status;        /* [b] PV_PNP_STOP_* */
    double *cost;           /* [b] final 0.5 * sum r^2 */
} pv_pnp_diag;

#define PV_PNP_STOP_GRADIENT 1
#define PV_PNP_STOP_PARAMETER 2
#define PV_PNP_STOP_FUNCTION 3
#define PV_PNP_STOP_MAX_ITER 4
#define PV_PNP_STOP_RADIUS 5
#define PV_PNP_STOP_P3P_ONLY 6  /* pn == 4: the P3P pose is the result (extend_utils.py:90-94) */

/* replaces extend_utils.uncertainty_pnp / uncertainty_pnp_v2 (extend_utils.py:63-166): per image the
 * P3P pose of the four highest-weight points (cv2.solvePnP SOLVEPNP_P3P: points 0..2 solve, point 3
 * picks), then the weighted reprojection least squares of src/uncertainty_pnp.cpp:7-92 by Ceres 2.0's
 * Levenberg-Marquardt (restated).  Rt out f64 [b][3][4] = [Rodrigues(r) | t].  One wave per
 * image, fp64. */
int pv_uncertainty_pnp(const pv_pnp_batch *batch, double *Rt, const pv_pnp_diag *diag, pv_stream_t stream);

/* replaces the C entry uncertainty_pnp(pts2d, pts3d, wgt2d, K, init_rt, result_rt, pn)
 * (src/uncertainty_pnp.cpp:58-92): the least squares alone from given initial poses.
 * init_rt / result_rt f64 [b][6] (angle-axis, translation); mode must be PV_PNP_WEIGHTS. */
int pv_uncertainty_pnp_refine(const pv_pnp_batch *batch, const double *init_rt, double *result_rt,
                              const pv_pnp_diag *diag, pv_stream_t stream);

/* ---- the network's decoder (the ResNet-18 seg + vector-field forward, A8) ---- */

/* replaces nn.UpsamplingBilinear2d(scale_factor=2) followed by torch.cat([up(fm), skip], 1)
 * (lib/networks/model_repository.py:35-51 modules, :66-75 forward) for channels-last fp16 maps, fused
 * into one pass, with channels [c1 + c2, cpad) of the output zero (a pad for the convolution after it).
 * x: [n][hin][win][c1] fp16 (a channels_last NCHW tensor's memory), skip: [n][2 hin][2 win][c2] (may be
 * NULL when c2 = 0), out: [n][2 hin][2 win][cpad].  c1 and cpad multiples of 8, cpad >= c1 + c2, x and
 * out 16-byte aligned.  The blend is ATen's upsample_bilinear2d (align_corners=True) arithmetic in f32. */
int pv_upsample2x_cat_f16(const void *x, const void *skip, void *out, int32_t n, int32_t hin, int32_t win,
                          int32_t c1, int32_t c2, int32_t cpad, pv_stream_t stream);
/* the same for f32 maps: c1 and cpad multiples of 4 */
int pv_upsample2x_cat_f32(const void *x, const void *skip, void *out, int32_t n, int32_t hin, int32_t win,
                          int32_t c1, int32_t c2, int32_t cpad, pv_stream_t stream);

/* replaces, for channels-last maps, the passes the reference's modules make after each convolution
 * (lib/networks/resnet.py:41-70 BasicBlock: bn -> relu, bn + residual -> relu; model_repository.py:22-58:
 * bn -> ReLU / LeakyReLU(0.1); :66-67 the torch.cat after fc), with the BatchNorm folded into a bias:
 * out[p][0:c1] = act(x[p] + bias (+ (res[p] + rbias))), out[p][c1:c1+c2] = skip[p], in one pass.
 * x, res: [P][c1]; skip: [P][c2] (NULL when c2 = 0); bias, rbias: [c1] (rbias may be NULL);
 * out: [P][c1 + c2] (may be x itself when c2 = 0).  act PV_ACT_*; slope for PV_ACT_LEAKY.
 * fp16: c1, c2 multiples of 8; f32: of 4; all pointers 16-byte aligned.  Roundings as ATen's unfused ops. */
#define PV_ACT_NONE 0
#define PV_ACT_RELU 1
#define PV_ACT_LEAKY 2
int pv_conv_epilogue_f16(const void *x, const void *bias, const void *res, const void *rbias, const void *skip,
                         void *out, int64_t P, int32_t c1, int32_t c2, int32_t act, float slope, pv_stream_t stream);
int pv_conv_epilogue_f32(const void *x, const void *bias, const void *res, const void *rbias, const void *skip,
                         void *out, int64_t P, int32_t c1, int32_t c2, int32_t act, float slope, pv_stream_t stream);

/* replaces the stem's tail (lib/networks/resnet.py:201-204: relu(bn1(conv1(x))) = x2s, then
 * maxpool 3x3 / stride 2 / pad 1) for channels-last maps, BN folded into bias: x2s = relu(x + bias)
 * [n][h][w][c] and pool = maxpool(x2s) [n][(h-1)/2+1][(w-1)/2+1][c] in one pass.  x: the convolution's
 * output without bias; bias [c]; fp16: c a multiple of 8, f32: of 4; pointers 16-byte aligned, the three
 * maps distinct.  Both outputs equal ATen's bias add + ReLU + max_pool2d bit for bit.  bias and x2s
 * both NULL: pool-only (x is x2s already, e.g. from pv_stem_conv_f16). */
int pv_relu_maxpool_f16(const void *x, const void *bias, void *x2s, void *pool, int32_t n, int32_t h, int32_t w,
                        int32_t c, pv_stream_t stream);
int pv_relu_maxpool_f32(const void *x, const void *bias, void *x2s, void *pool, int32_t n, int32_t h, int32_t w,
                        int32_t c, pv_stream_t stream);

/* replaces the stem's convolution (lib/networks/resnet.py:139-142, 201-203: conv1 7x7 / stride 2 /
 * pad 3, 3 -> 64 channels, bn1 folded into w / bias, relu) for a channels-last fp16 batch:
 * img [n][h][wd][3] (h, wd even, 4-byte aligned), out = x2s [n][h/2][wd/2][64] (16-byte aligned).
 * w: the folded weights in the kernel's space-to-depth layout [2][16 taps (ty, tx)][2][32][8] fp16
 * (pvnet_amd.network.stem_weights: tap (ty, tx) channel dy*6 + dx*3 + c = W[c][2ty+dy-1][2tx+dx-1]),
 * bias [64] fp16.  Roundings: the f32 sum rounded to fp16, + bias, ReLU (as ATen's conv then bias
 * add and relu; the sum's order differs from MIOpen's). */
int pv_stem_conv_f16(const void *img, const void *w, const void *bias, void *out, int32_t n, int32_t h, int32_t wd,
                     pv_stream_t stream);
/* the same convolution and, from the same pass, the maxpool after it (lib/networks/resnet.py:204:
 * 3x3 / stride 2 / pad 1): x2s as above, pool [n][(h/2 - 1)/2 + 1][(wd/2 - 1)/2 + 1][64] (16-byte
 * aligned) = max over each window of x2s (bit-equal to max_pool2d of x2s). */
int pv_stem_pool_f16(const void *img, const void *w, const void *bias, void *x2s, void *pool, int32_t n, int32_t h,
                     int32_t wd, pv_stream_t stream);

/* replaces, for layer1's convolutions (lib/networks/resnet.py:21-70 BasicBlock conv1 / conv2 at
 * 64 -> 64 channels, 3x3, stride 1, pad 1), MIOpen's convolution + the epilogue pass after it:
 * out = act(conv(x) + bias (+ res)), fp16 channels-last, x / res / out [n][h][wd][64].  w: the folded
 * weights as [9 taps (ky, kx)][8 octets q][64 couts][8] fp16 = W[cout][8q + j][ky][kx]
 * (pvnet_amd.network.conv64_weights), bias [64].  act: PV_ACT_NONE or PV_ACT_RELU.  x, w, res, out
 * 16-byte, bias 8-byte aligned; out distinct from x and res.  Roundings as pv_conv3x3_f16. */
int pv_conv64_f16(const void *x, const void *w, const void *bias, const void *res, void *out, int32_t n, int32_t h,
                  int32_t wd, int32_t act, pv_stream_t stream);

/* replaces convraw's tail (model_repository.py:53-58 after the 3x3 convolution): BN bias + LeakyReLU(slope)
 * + the 1x1 convolution to seg_dim + ver_dim channels with its bias, one pass.  x: [P][cin] channels-last
 * (the 3x3 convolution's output without bias), b1 f32 [cin], w2 f32 [cout][cin], b2 f32 [cout] (device),
 * out: [P][cout].  (cin, cout) = (32, 20) or (32, 44); x 16-byte, out 8-byte aligned. */
int pv_head_f16(const void *x, const float *b1, const float *w2, const float *b2, void *out, int64_t P,
                int32_t cin, int32_t cout, float slope, pv_stream_t stream);
int pv_head_f32(const void *x, const float *b1, const float *w2, const float *b2, void *out, int64_t P,
                int32_t cin, int32_t cout, float slope, pv_stream_t stream);

/* replaces, for the backbone's wide 3x3 convolutions (lib/networks/resnet.py:21-38 conv3x3 with
 * dilation, :167-198 layer2 / layer3 / layer4; model_repository.py:22-35 fc, conv8s), MIOpen's convolution + the
 * epilogue pass after it: out = act(conv(x) + bias (+ (res + rbias))), fp16, channels-last, stride 1,
 * padding = dilation.  x [n][h][w][cin], w [cout][3][3][cin] (the conv weight permuted; BN folded),
 * bias / rbias [cout], res [n][h][w][cout], out [n][h][w][ldo] (channels [0, cout) written; ldo = 0:
 * cout -- ldo > cout writes into a wider map, e.g. the torch.cat after fc, MR:66).  res, rbias may be
 * NULL.  cin a multiple of 64, cout of 128, ldo of 4; x, w, res, out 16-byte, bias, rbias 8-byte
 * aligned; out distinct from x and res.  act PV_ACT_*.  The sums are f32 (matrix cores) rounded to fp16,
 * then pv_conv_epilogue's roundings. */
int pv_conv3x3_f16(const void *x, const void *w, const void *bias, const void *res, const void *rbias, void *out,
                   int32_t ldo, int32_t n, int32_t h, int32_t wd, int32_t cin, int32_t cout, int32_t dil,
                   int32_t act, float slope, pv_stream_t stream);

/* pv_conv3x3_f16 generalised to the rest of the backbone's 3x3 convolutions (lib/networks/resnet.py:
 * 21-70 BasicBlock with its downsample, :167-198 layer2's stride-2 first block; model_repository.py:
 * 22-35,66 fc -> torch.cat([xfc, x8s], 1) -> conv8s):
 *   x [n][hin][win][cin] read at stride `stride` (1 or 2; padding = dilation, so h = (hin - 1) / stride
 *   + 1, wd likewise);
 *   mode2 PV_CONV_X2_CAT: x2 [n][hin][win][cin2] is the concatenation's second part -- the 3x3
 *   convolution runs over cat([x, x2]) (w [cout][3][3][cin + cin2]) without the concatenated map;
 *   mode2 PV_CONV_X2_1X1: x2 [n][h2][w2][cin2] feeds a 1x1 convolution at stride s2 summed into the
 *   same accumulator (the BasicBlock's downsample, its weight appended: w [cout][9 cin + cin2]);
 *   rbias (its bias, res NULL) is added after the bias, before the activation.
 * ws (256-byte aligned, ws_bytes from pv_conv3x3_workspace_bytes(n h wd, cout, K-steps), or NULL): the
 * scratch that lets the launch cut its last partial round of 256-pixel tiles (tiles mod CUs) into K
 * parts run side by side, the last-arriving part summing the others' f32 partials in part order (the
 * result does not depend on the arrival order); K-steps = 9 (cin + cin2 for PV_CONV_X2_CAT) / 64
 * (+ cin2 / 64 for PV_CONV_X2_1X1).  ws must be zero-filled before its first use; every call leaves
 * it so.  One ws per stream at a time.
 * Other arguments, alignment and roundings as pv_conv3x3_f16 (which is this with stride 1,
 * PV_CONV_X2_NONE and no ws). */
#define PV_CONV_X2_NONE 0
#define PV_CONV_X2_CAT 1
#define PV_CONV_X2_1X1 2
int pv_conv3x3_ex_f16(const void *x, int32_t hin, int32_t win, int32_t stride, const void *x2, int32_t mode2,
                      int32_t cin2, int32_t h2, int32_t w2, int32_t s2, const void *w, const void *bias,
                      const void *res, const void *rbias, void *out, int32_t ldo, int32_t n, int32_t h,
                      int32_t wd, int32_t cin, int32_t cout, int32_t dil, int32_t act, float slope, void *ws,
                      int64_t ws_bytes, pv_stream_t stream);
int64_t pv_conv3x3_workspace_bytes(int64_t pixels, int32_t cout, int32_t ksteps);
/* the leading bytes of that ws that hold its arrival counters (the part that must start zeroed; the
 * rest is overwritten before it is read): a scratch made inside a graph capture zeroes only these.
 * The same 4 KiB for every shape that splits, so one ws serves calls of any shapes in turn. */
int64_t pv_conv3x3_workspace_counter_bytes(int64_t pixels, int32_t cout, int32_t ksteps);

/* replaces the decoder's half-resolution step (model_repository.py:43-51,75-78: up4sto2s, torch.cat([fm,
 * x2s], 1), conv2s = 3x3 conv + BN + LeakyReLU(slope)) in one fp16 matrix-core pass: fm [n][hin][win][64]
 * (conv4s's output), skip [n][2hin][2win][64] (x2s), out [n][2hin][2win][32], all channels-last.  w: the
 * 3x3 weights with BN folded, laid out [2][9][8][32][8] fp16: element [p][3 ky + kx][q][cout][j] =
 * W[cout][64 p + 8 q + j][ky][kx] (p = 0 the upsampled channels, 1 the skip); bias fp16 [32].  fm, skip,
 * w, out 16-byte, bias 8-byte aligned.  Roundings as pv_decoder_tail_f16's blend and convolution, then
 * the bias add and LeakyReLU as ATen. */
int pv_decoder_conv2s_f16(const void *fm, const void *skip, const void *w, const void *bias, void *out, int32_t n,
                          int32_t hin, int32_t win, float slope, pv_stream_t stream);

/* replaces the decoder's quarter-resolution step (model_repository.py:35-43,75-77: up8sto4s, torch.cat([fm,
 * x4s], 1), conv4s = 3x3 conv + BN + LeakyReLU) in one fp16 matrix-core pass: fm [n][hin][win][128]
 * (conv8s's output), skip [n][2hin][2win][64] (x4s), out [n][2hin][2win][64].  w: [3][9][8][2][32][8] fp16,
 * element [p][3 ky + kx][q][m][c][j] = W[32 m + c][64 p + 8 q + j][ky][kx] (p = 0, 1 the upsampled channels,
 * 2 the skip); bias fp16 [64].  Alignment and roundings as pv_decoder_conv2s_f16. */
int pv_decoder_conv4s_f16(const void *fm, const void *skip, const void *w, const void *bias, void *out, int32_t n,
                          int32_t hin, int32_t win, float slope, pv_stream_t stream);

/* replaces the decoder's full-resolution tail (model_repository.py:75-79: up2storaw, torch.cat([fm, x], 1),
 * convraw = 3x3 conv + BN + LeakyReLU(slope) + 1x1 conv) in one fp16 pass on the matrix cores:
 * fm [n][hin][win][32] (conv2s's output, channels-last), img [n][2hin][2win][3] (the input batch,
 * channels-last), out [n][2hin][2win][cout], cout = 20 or 44.  w1: [32][368] fp16, the 3x3 weights with
 * BN folded, k = (3 ky + kx) * 40 + input channel (channels 35..39 and k >= 360 zero); b1 f32 [32];
 * w2: [cout/32 rounded up][2][32][16] fp16, the 1x1 weights in the accumulator's row order
 * (element [t][s][m][8h + j] = W[32t + m][(j & 3) + 8 (j >> 2) + 16 s + 4 h], zero past cout); b2 f32
 * [cout].  fm, w1, w2 16-byte, out 8-byte aligned.  Roundings: the 3x3 sums to fp16 (as a fp16
 * convolution's output), then ATen's bias add and LeakyReLU, the 1x1 sums to fp16, then its bias add. */
int pv_decoder_tail_f16(const void *fm, const void *img, const void *w1, const float *b1, const void *w2,
                        const float *b2, void *out, int32_t n, int32_t hin, int32_t win, int32_t cout, float slope,
                        pv_stream_t stream);
/* pv_decoder_tail_f16 with the head's output split the way the network returns it (model_repository.py:79:
 * seg_pred = x[:, :seg_dim], ver_pred = x[:, seg_dim:], seg_dim = 2): seg [n][2hin][2win][2] and ver
 * [n][2hin][2win][cout - 2], each channels-last and dense, so the voting layer's argmax reads 4 bytes per
 * pixel instead of the whole cout-channel record's cache lines.  The same values as pv_decoder_tail_f16's
 * channels.  seg, ver 4-byte aligned. */
int pv_decoder_tail_split_f16(const void *fm, const void *img, const void *w1, const float *b1, const void *w2,
                              const float *b2, void *seg, void *ver, int32_t n, int32_t hin, int32_t win,
                              int32_t cout, float slope, pv_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* PVVOTE_H_ */
