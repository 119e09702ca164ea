// Host-side launch API of the fused ResNet-20 kernels (csrc/kernels/resnet.hip).
//
// Conventions: activations NHWC bf16; per-layer BatchNorm statistics live in NSLOT fixed-point slots
// per layer (slot = producing block & 7; int64 [NSLOT][hi 128 | lo 128], integer part + 48-bit
// fraction added with 64-bit integer atomics -- order independent, so bitwise reproducible; zeroed
// once per step by the engine).  Conv weights have two bf16 shadows:
//   fwd   w [COUT][KP]  k  = tap*CINP + ci        (tap = kh*3 + kw, CINP = max(CIN, 8), KP = 9*CINP -> x32)
//   dgrad wd [CIN][KPD] k' = tap'*COUT + co       (tap' = 8 - tap: rotated 180 degrees, KPD = 9*COUT -> x32)
// Layer l computes z_l = conv_l(x_l) with x_l = a_{l-1}, a = relu(bn(z) [+ shortcut]).
// Any batch size: the kernels run on B (a multiple of 16) images, the first `nvalid` real; the padding
// images are excluded from every BatchNorm statistic (inv_n = 1 / (nvalid * H * W)) and get exactly zero
// loss weight and gradient, so the step equals the eager model's at batch nvalid.
#pragma once
#include "api.h"

extern "C" {

struct DmlcRnLayerGeom {    // runtime copy of the compile-time geometry (validated by the binding)
  int cin, cout, hin, stride;
  int per_image;             // rn_bwd: one workgroup per image for dgrad AND wgrad (16->16 layers, G == B)
};

struct DmlcRnFwdArgs {
  // input of this conv: the dataset (stem) or the BN-apply of the previous layer
  const uint8_t* data; DmlcIndexSrc src; int cy, cx;      // stem only
  const void* z_prev;        // bf16 [B][Hin][Hin][CIN]  pre-BN output of layer l-1
  const long long* stat_prev;   // [NSLOT][256] fixed-point sum z, sum z^2 of layer l-1
  const float* gamma_prev; const float* beta_prev;
  const void* sc_src;        // nullable: block input feeding the residual of layer l-1 (bf16)
  int sc_mode;               // 0 none, 1 identity [B][Hin][Hin][CIN], 2 subsample+zero-pad [B][2Hin][2Hin][CIN/2]
  void* a_out;               // bf16 [B][Hin][Hin][CIN]  materialised a_{l-1} (backward needs it)
  float inv_n_prev;          // 1 / (B * Hin * Hin)
  const void* w;             // bf16 [COUT][KP]
  void* z;                   // bf16 [B][Hout][Hout][COUT]
  long long* stat;           // [NSLOT][256] fixed-point accumulators of layer l
  int B;
  int nvalid;                // images b >= nvalid are batch padding: no contribution to the statistics
};

struct DmlcRnDgradArgs {
  // BN backward of layer l (prologue): g_z = gamma*rstd*(g_y - R1/N - xhat*R2/N)
  const void* gy; const void* z; const long long* stat; const long long* red; const float* gamma; float inv_n;
  const void* wd;            // bf16 [CIN][KPD]
  // epilogue: g_a_{l-1} (+ shortcut) -> g_y_{l-1} = g_a * (a_{l-1} > 0), reductions of layer l-1
  const void* a_prev; const void* z_prev; const long long* stat_prev; float inv_n_prev;
  const void* gy_sc;         // nullable: g_y of the block's second conv (shortcut gradient)
  int sc_mode;               // 1 identity, 2 subsample (gy_sc is [B][Hin/2][Hin/2][2*CIN])
  void* gy_prev;             // bf16 [B][Hin][Hin][CIN]
  long long* red_prev;       // [NSLOT][256]
  int B;
  int nvalid;                // padding images (b >= nvalid) get g_z = 0 (their g_y is 0 already)
};

struct DmlcRnWgradArgs {
  const uint8_t* data; DmlcIndexSrc src; int cy, cx;      // stem input
  const void* x;             // bf16 a_{l-1} [B][Hin][Hin][CIN] (l >= 1)
  const void* gy; const void* z; const long long* stat; const long long* red; const float* gamma; float inv_n;
  float* part;               // [G][KP][COUT] fp32 split-K slabs
  int G, B;
  int nvalid;                // padding images contribute nothing (g_z = 0)
};

struct DmlcRnHeadArgs {
  const void* z; const long long* stat; const float* gamma; const float* beta; float inv_n;   // layer 18
  const void* sc;            // identity shortcut (block input) bf16 [B][8][8][64]
  const float* fcw; const float* fcb;   // fp32 master views [64][10], [10]
  const int* labels; DmlcIndexSrc src; float inv_batch;
  void* gy;                  // bf16 [B][8][8][64] g_y_18
  long long* red;            // [NSLOT][256] reductions of layer 18
  float* fc_part;            // [B][656] per-image dW_fc (640) + db_fc (10) + pad
  float* loss_img; int* correct_img;    // [B]
  float* logits_out;         // nullable [B][10]
  int B;
  int nvalid;                // images b >= nvalid: no loss, no accuracy, zero gradient
  const int64_t* step; int64_t* step_copy;   // nullable: workgroup 0 copies *step (read by the SGD)
};

#define DMLC_RN_LAYERS 19
#define DMLC_RN_NSLOT 8      // fixed-point statistics slots per layer: [NSLOT][256] int64 (slot = block & 7)
struct DmlcRnSgdArgs {
  float* master; int nparams;
  float* grad; float grad_scale;   // DP: modes 1 (write) / 2 (read, scaled)
  // per conv layer
  int conv_off[DMLC_RN_LAYERS], gamma_off[DMLC_RN_LAYERS], beta_off[DMLC_RN_LAYERS];
  int cin[DMLC_RN_LAYERS], cout[DMLC_RN_LAYERS];
  const float* part[DMLC_RN_LAYERS]; int G[DMLC_RN_LAYERS];
  void* wf[DMLC_RN_LAYERS]; void* wd[DMLC_RN_LAYERS];
  const long long* stat; const long long* red;   // [19][NSLOT][256] each
  float* state; int mm_off[DMLC_RN_LAYERS], mv_off[DMLC_RN_LAYERS];   // BN moving statistics
  float bn_momentum; float inv_n[DMLC_RN_LAYERS];
  int fcw_off, fcb_off; const float* fc_part; int B;
  int blk_start[DMLC_RN_LAYERS + 3];   // block ranges (set by the launcher): conv layers, fc, BN layers
  int split[DMLC_RN_LAYERS + 1];       // slab split factor per conv layer + fc (set by the launcher)
  int mode;                  // 0 reduce+apply, 1 reduce->grad, 2 apply grad, 3 shadows only
  // conv layers [layer_lo, layer_hi) only; tail = also the fc / BN parameters, the BN running
  // statistics and the step publication (a partial launch of the conv layers whose weight gradients
  // are complete can run on a graph branch beside the rest of the backward)
  int layer_lo, layer_hi, tail;
  int64_t* step; float lr0, decay, decay_steps; int staircase;
  float warmup;             // linear LR warm-up steps (0: none)
  unsigned int* ticket;
  const int64_t* step_rd;   // == step (ticket: the last arriver bumps it) or the head's copy (the BN
                            // layer-0 block bumps it, no ticket)
  const float* loss_img; const int* correct_img;
  float* stats; int stats_len;
  int nvalid;                // valid images of the batch (loss / accuracy means)
};

hipError_t dmlc_rn_fwd(const DmlcRnLayerGeom* g, const DmlcRnFwdArgs* a, hipStream_t s);
hipError_t dmlc_rn_dgrad(const DmlcRnLayerGeom* g, const DmlcRnDgradArgs* a, hipStream_t s);
hipError_t dmlc_rn_wgrad(const DmlcRnLayerGeom* g, const DmlcRnWgradArgs* a, hipStream_t s);
// dgrad (workgroups [0, B)) + wgrad (the rest) of one layer in one launch
hipError_t dmlc_rn_bwd(const DmlcRnLayerGeom* g, const DmlcRnDgradArgs* d, const DmlcRnWgradArgs* w, hipStream_t s);
hipError_t dmlc_rn_head(const DmlcRnHeadArgs* a, hipStream_t s);
hipError_t dmlc_rn_sgd(DmlcRnSgdArgs* a, hipStream_t s);

}  // extern "C"
