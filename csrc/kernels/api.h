// Host-side launch API of the HIP CNN kernels.
//
// Plain C structs + launch functions so that the torch binding TU (compiled by g++) never sees
// device code, and the kernel TUs (compiled by hipcc) never include torch headers.
// Every pointer is device memory; bf16 tensors are passed as `const void*` / `void*`.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// uints in the arrival-ticket buffer of the SGD launches (two-level counters, common.h last_arrival)
#define DMLC_TICKET_WORDS (9 * 32)

extern "C" {

// Batch index source shared by the data-consuming kernels.  Two forms:
//  * explicit list (idx_base != null): sample of row b is
//      idx_base[(counter ? (*counter % period) : 0) * B + b]
//  * generated order (idx_base == null, counter required): the training order is a keyed Feistel
//    bijection of [0, n) per epoch (common.h order_index; dmlc/data/order.py is the host twin).
//    With s = *counter, epoch = s / period, j = s % period, row b < bvalid of rank r reads
//      perm_epoch((j * world + r) * bvalid + b)
//    so a captured graph crosses epoch boundaries with no host work, and the W ranks of a step
//    read exactly the rows a single rank with batch W*bvalid would.  Rows b >= bvalid (padding up
//    to the kernel tile) read row bvalid - 1; their loss gradient is zeroed by the head.
struct DmlcIndexSrc {
  const int* idx_base;      // nullable: generated order
  const int64_t* counter;   // nullable (explicit list only)
  int period;               // explicit: B-sized batches in idx_base; generated: steps per epoch
  int n, half_bits, world, rank, bvalid;
  uint32_t seed;
};

// conv1 5x5 (3->64) + bias + ReLU + maxpool 3x3/2 TF-SAME, fused with the uint8 gather + center
// crop.  One workgroup per image.
struct DmlcConv1FwdArgs {
  const uint8_t* data;      // [N][32][32][3] uint8 (NHWC)
  DmlcIndexSrc src;
  int B, cy, cx;            // crop offsets (center crop = 4,4)
  const void* w;            // bf16 [64][96]  (k = kh*16 + kw*3 + ci, zero padded)
  const float* bias;        // [64]
  void* out;                // bf16 [B][12][12][64]
  uint8_t* am;              // [B][12][12][64] argmax (0..8) in the pool window, 255 = no gradient
  float* amax;              // nullable: fp8 path, float[B] per-image max of the pooled output (plain
                            //   stores, no atomics; the fp8 conv2 forward reduces them)
  uint8_t* xraw;            // nullable: copy of each row's raw uint8 image [B][3072] for the wgrad
  int xraw_in;              // k_conv12_fwd: read row b's image from xraw[b] (written for this step by
                            //   the previous step's finalizer), no index load, no copy-out
};

// conv2 5x5 (64->64) + bias + ReLU + maxpool 3x3/2 TF-SAME.  One workgroup per image.
struct DmlcConv2FwdArgs {
  const void* in;           // bf16 [B][12][12][64]
  const void* w;            // bf16 [64 co][1600]  (k = (kh*5+kw)*64 + ci)
  const float* bias;        // [64]
  void* out;                // bf16 [B][6][6][64]  (== [B][2304], NHWC flatten order)
  uint8_t* am;              // [B][6][6][64]
  int B;
};

// conv2 forward on fp8 (OCP e4m3fn) MFMA operands, per-tensor scales (BASELINE config 5).
// x8 = sat(x * 448 / max_b amax_x[b]), w8 = w2f8 (quantised by the SGD kernel with scale_w[step&1]);
// out = relu(acc / (sx * sw) + b), then the same TF-SAME pool as the bf16 path.
struct DmlcConv2FwdFp8Args {
  const void* in;           // bf16 [B][12][12][64]
  const uint8_t* w8;        // fp8 [64 co][1600]
  const float* bias;        // [64]
  const float* amax_x;      // float[B] (conv1 pool output max per image, this batch)
  const float* scale_w;     // float[2] (weight quantisation scale, slot step & 1)
  const int64_t* counter;   // device global_step (nullable: slot 0)
  void* out;                // bf16 [B][6][6][64]
  uint8_t* am;              // [B][6][6][64]
  int B;
  uint8_t* x8out;           // nullable: the quantised input e4m3 [B][144][64] (the fp8 weight gradient's X)
  float* sx_out;            // nullable (with x8out): its per-batch scale sx, float[1]
};

// conv2 input gradient on fp8 MFMA operands (BASELINE config 5 backward): w8 = the flipped, ci-major
// W2 (w2d layout) quantised with scale_w (the SGD kernel writes it next to w2f8, both scale slots
// hold the current scale); dY2 quantised per image in-kernel.  Outputs as DmlcConv2DgradArgs.
struct DmlcConv2DgradFp8Args {
  const void* dp2;          // bf16 [B][6][6][64]
  const uint8_t* am2;       // [B][6][6][64]
  const uint8_t* w8;        // fp8 [64 ci][1600]  (k' = (kh'*5+kw')*64 + co, W[4-kh'][4-kw'][ci][co] * sw)
  const float* scale_w;     // float[2]
  void* dp1;                // bf16 [B][12][12][64]
  void* dy2;                // bf16 [B][144][64]
  int B;
  uint8_t* dy8out;          // nullable: the quantised dY2 e4m3 [B][144][64] (the fp8 weight gradient's dY)
  float* sy_img;            // nullable (with dy8out): float[B], image b's power-of-two dY2 scale
};

// conv2 input-gradient with the pool2/ReLU backward fused into the operand staging.
struct DmlcConv2DgradArgs {
  const void* dp2;          // bf16 [B][6][6][64]  grad wrt pool2 output
  const uint8_t* am2;       // [B][6][6][64]
  const void* wd;           // bf16 [64 ci][1600]  (k' = (kh'*5+kw')*64 + co, W[4-kh'][4-kw'][ci][co])
  void* dp1;                // bf16 [B][12][12][64] grad wrt pool1 output
  void* dy2;                // bf16 [B][144][64]   grad wrt conv2 pre-activation (for wgrad)
  int B;
  int split;                // in the fc chain: 2 workgroups per image (B <= 128), else one
};

// conv1 weight gradient (pool1/ReLU backward fused; split-K over image groups).
struct DmlcConv1WgradArgs {
  const uint8_t* data;      // [N][32][32][3]
  DmlcIndexSrc src;
  const uint8_t* xraw;      // nullable: the forward's copy [B][3072] (row b) instead of data[src(b)]
  int cy, cx;
  const void* dp1;          // bf16 [B][12][12][64]  grad wrt pool1 output
  const uint8_t* am1;       // [B][12][12][64]
  float* part1;             // [g1][80][64]  k'' = kh*16 + kw*3 + ci (k'' % 16 == 15 unused)
  float* partb1;            // [g1][64]
  int g1;
  int B;
};

// conv2 weight gradient: blocks (input-channel quarter, image group); fp32 partial slab per group.
struct DmlcConv2WgradArgs {
  const void* p1;           // bf16 [B][12][12][64]   (conv2 input)
  const void* dy2;          // bf16 [B][144][64]      (conv2 pre-activation gradient)
  void* part2;              // [g2][1600][64] fp32
  float* partb2;            // [g2][64] conv2 bias-grad partials (written by the c4 == 0 blocks)
  int g2;
  int B;
  // fp8 (BASELINE config 5): the conv2 weight gradient on v_mfma_scale_f32_16x16x128_f8f6f4 over the
  // e4m3 copies the fp8 forward (X, per-batch scale sx) and the fp8 dgrad (dY2, a power-of-two scale
  // per image, applied as the MFMA's E8M0 block scale) wrote; x8 == null: bf16 MFMA on p1 / dy2
  const uint8_t* x8;        // e4m3 [B][144][64]
  const uint8_t* y8;        // e4m3 [B][144][64]
  const float* sx;          // float[1]
  const float* sy_img;      // float[B]
};


// Grouped bf16 GEMM: up to 8 independent problems in one launch, 64x64 tiles, MFMA 16x16x32.
//   a_kmajor=1: A(m,k) = A[m*lda + k]; 0: A(m,k) = A[k*lda + m]
//   b_kmajor=1: B(k,n) = B[n*ldb + k]; 0: B(k,n) = B[k*ldb + n]
//   c_mode 0: fp32 C[m*ldc+n] (+bias, relu)  1: bf16 C (+bias, relu)
//          2: fp32 split-K partial slab C + split*M*ldc   3: column sums: C[m] = sum_k A(m,k), m < nvalid
struct DmlcGemmProblem {
  int M, N, K;
  const void* A; int lda; int a_kmajor;
  const void* B; int ldb; int b_kmajor;
  void* C; int ldc; int c_mode;
  int ksplit;
  const float* bias; int relu;
  int nvalid;               // store only columns n < nvalid
  // step-parity double buffers (G.step): b_par != 0 -> the B operand is B + b_par elements on odd
  // steps; c_mode 4 (fused SGD, fp32 C = the master weights): w -= lr(step) * grad_scale * acc, and
  // the bf16 shadow of the NEXT step goes to S + (step+1 odd ? s_par : 0) at the same [m][ldc] offsets
  long long b_par, s_par;
  void* S;
  int tiles_m, tiles_n, block_start;   // filled by dmlc_gemm_grouped
};
#define DMLC_MAX_GEMM 8
struct DmlcGemmGroup {
  DmlcGemmProblem p[DMLC_MAX_GEMM];
  int nprob;
  int nblocks;
  // device step counter (nullable: parity 0) and the SGD schedule for c_mode 4 (same as DmlcSgdArgs)
  const int64_t* step;
  float lr0, decay, decay_steps, warmup, grad_scale;
  int staircase;
  // XCD-aware tile order: every problem's block range is padded to a multiple of 8 and XCD x
  // (= blockIdx % 8 under round-robin dispatch) takes a contiguous 1/8 of its tiles, so the blocks
  // that share the larger operand's tiles (or, split-K, one K slice) share an L2 (speed only)
  int xcd_map;
};

// MLP head, rows-parallel (rows = 2 or 4 per workgroup; B / rows workgroups): fc1 split-K reduce + bias + ReLU, fc2, fc3,
// (ReLU logits), softmax cross-entropy + accuracy, and (train) the backward through fc3/fc2.
struct DmlcHeadArgs {
  const float* h1part; int nsplit;   // [nsplit][B][384]
  const float* b1;
  const void* w2t; const float* b2;  // bf16 [192][384]
  const void* w3t; const float* b3;  // bf16 [16][192] (rows >= 10 zero)
  const void* w3d;                   // bf16 [192][32] (cols >= 10 zero)
  const void* w2d;                   // bf16 [384][192]
  const int* labels;                 // [N] dataset labels
  DmlcIndexSrc src;
  int B; int rows; float inv_batch; int relu_logits; int train;
  int nvalid;                        // rows b >= nvalid are padding: no loss, accuracy or gradient
  void* h1; void* h2; void* dl; void* dh1; void* dh2;   // bf16 [B][384],[B][192],[B][16],[B][384],[B][192]
  float* loss_part; int* correct_part;                  // [B/rows]
  float* logits_out;                                    // optional fp32 [B][10]
  // optional: workgroup 0 copies *step to *step_copy -- the value the step's SGD launch reads, so
  // the SGD can bump *step from any one block without an arrival ticket (no SGD block reads *step)
  const int64_t* step; int64_t* step_copy;
};

// The fully-connected part of a training step in ONE persistent launch (cnn_fc.hip; B <= 256,
// B % 16 == 0; 256 co-resident workgroups): fc1 forward (split-K), the MLP head (loss, accuracy,
// dlogits -> dh2 -> dh1), and the fc backward (dp2 = dh1 W1^T, dW1 [+ fused fc1 SGD], dW2, dW3, db).
struct DmlcFcArgs {
  int B, nvalid, mtiles;             // padded batch, real rows, ceil(B / 64)
  const void* p2;                    // bf16 [B][2304] pooled conv2 output (NHWC flatten)
  void* w1;                          // bf16 [2][2304][384] fc1 shadow (step parity; fused SGD writes the other)
  float* h1part;                     // fp32 [8][B][384] fc1 split-K partials (workspace)
  const float* b1;
  const void* w2t; const float* b2;  // bf16 [192][384]
  const void* w3t; const float* b3;  // bf16 [16][192]
  const void* w3d;                   // bf16 [192][32]
  const int* labels;
  DmlcIndexSrc src;
  float inv_batch; int relu_logits;
  void* h1; void* h2; void* dl; void* dh1; void* dh2;   // bf16 hand-off rows (as DmlcHeadArgs)
  float* loss_part; int* correct_part;                  // [B / 4]
  void* dp2;                         // bf16 [B][2304] out: the conv backward's input
  float* gw1;                        // fuse_sgd: fc1 fp32 master (updated); else the fc1 weight gradient
  float* gw2; float* gw3; float* gb1; float* gb2; float* gb3;   // gradients (flat grad views)
  // fuse_sgd: 0 every fc gradient to the flat gradient; 1 the fc1 weights updated in the dW1 epilogue
  // (gw1 = master), the rest gradients; 2 (the weight-gradient launch's apply mode) every fc
  // parameter updated in its dW epilogue: masters mw2 / mw3 / mb1..3 and the bf16 shadows below
  int fuse_sgd;
  float* mw2; float* mw3; float* mb1; float* mb2; float* mb3;
  void* fc2n; void* fc2t; void* fc3t; void* fc3d;   // bf16 [384][192], [192][384], [16][192], [192][32]
  int dw_tasks;                      // the fc-chain launch runs the dW tasks (0: the wgrad launch does)
  float lr0, decay, decay_steps, warmup, grad_scale; int staircase;
  const int64_t* step; int64_t* step_copy;             // device step counter; copy for the SGD reader
  unsigned int* sync;                // >= 28 * 32 zeroed uints (counters re-arm themselves)
  unsigned int* err;                 // sticky error word (value 2 = bit 1: a seam wait timed out)
  int grad_bf16;                     // fuse_sgd 0: gw1..gb3 are bf16 views (DmlcSgdArgs::grad16)
};

// Fused SGD over the flat fp32 parameter buffer (+ split-K partial reduction, LR schedule from the
// device step counter, bf16 shadow-weight refresh, step++ by the last workgroup, stats ring).
struct DmlcSgdArgs {
  float* master;            // flat fp32 params (TF layouts)
  float* grad;              // flat fp32 grads (fc part written by the GEMMs)
  int mode;                 // 0 fused reduce+apply, 1 reduce only (conv grads -> grad), 2 apply from grad, 3 shadows only
  float grad_scale;         // applied to the gradient in modes 0/2 (1/world for averaged DP)
  // flat offsets of the 10 tensors, TF order
  int off[10];
  const float* part1; const float* partb1; int g1;   // conv1 partials [g1][80][64], [g1][64]
  const void* part2; int g2;                         // conv2 partials [g2][1600][64] fp32
  const float* partb2; int B;                        // conv2 bias partials [g2][64]
  // bf16 shadows
  void* w1f; void* w2f; void* w2d; void* fc1n; void* fc2t; void* fc2n; void* fc3t; void* fc3d;
  // schedule
  int64_t* step; float lr0; float decay; float decay_steps; int staircase;
  // the step this launch reads (LR, parity slots, stats): == step (then the last arriver of a ticket
  // bumps it), or the copy the head kernel made (then workgroup 0 bumps step, no ticket)
  const int64_t* step_rd;
  float warmup;             // linear LR warm-up over this many steps (0: none)
  unsigned int* ticket;     // zero-initialised arrival counter
  const float* loss_part; const int* correct_part; int nhead;
  float* stats; int stats_len;   // ring [stats_len][4] = {step, loss, accuracy, lr}
  int nblocks;
  // fp8 conv2 shadow (nullable).  amax_w = float[2][400]: slot s holds one maximum per conv2-row
  // block.  Modes 0/2 quantise the updated W2 with sw = 224 / max(amax_w[step&1][*]) (2x headroom
  // over the previous weights' amax), store sw to both scale_w slots and each block's new maximum to
  // amax_w[(step+1)&1][block] (plain stores).  Mode 3 uses slot step&1 (set by the host).
  uint8_t* w2f8; float* amax_w; float* scale_w;
  uint8_t* w2d8;            // nullable: fp8 [64 ci][1600] flipped shadow for the fp8 conv2 dgrad
  // block roles launched: 0 all, 1 conv rows + conv biases only, 2 fc only (data-parallel split of
  // the apply around the bucketed all-reduce); only launches with finalize = 1 bump global_step /
  // publish stats (their last arriver).
  int roles;
  int finalize;
  // next step's batch rows (nullable): the finalizing launch writes bidx[b] = the generated-order row
  // of batch row b at step+1 (next = the generated-order descriptor; its counter is unused), so the
  // data-consuming kernels of every step read ONE index per row (explicit list, period 1) instead of
  // evaluating the Feistel order themselves (~150 scalar instructions per row per wave).
  int* bidx; int bidx_n;
  DmlcIndexSrc next;
  // fc1n is [2][2304][384] (step-parity double buffer: kernels of step s read fc1n[s & 1]); modes
  // 0/2 write fc1n[(s+1) & 1], mode 3 fc1n[s & 1].  fc1_fused (mode 0): the fc1 WEIGHT update already
  // ran in the dW1 GEMM's epilogue (c_mode 4) -- the fc1 role covers the fc1 bias only
  int fc1_fused;
  // nullable: the finalizing launch also gathers the next step's raw images, xnext[b] = xdata[row of
  // batch row b at step+1] (3072 B each), so the next forward reads its image without the index
  // hop (DmlcConv1FwdArgs::xraw_in)
  uint8_t* xnext; const uint8_t* xdata;
  // nullable: the flat gradient in bf16 (data parallel over RCCL with the bf16 wire).  Then modes 1/2
  // write / read it instead of `grad` (null): the producers round once, the all-reduce runs on it in
  // place and the SGD reads it -- bitwise the fp32 gradient + cast + all-reduce + cast-back path,
  // without the two cast launches
  void* grad16;
};

// Both weight gradients in one launch (blocks [0,g1): conv1; then 4 * g2 conv2 blocks, one slab per group).
// apply = 1 (single GPU, cnn_wgrad.hip): the launch also finishes the step -- the blocks of each
// slab family meet at a sub-grid barrier (bar: DMLC_WBAR_WORDS zeroed uints), reduce their share of
// the slabs in the SGD kernel's order and apply the update (sgd: mode 0, fc1_fused, step_rd = the
// head's step copy); the conv1 blocks also run the fc roles, publish the stats and bump global_step.
// No SGD launch follows.  bar[10 * 32] is a sticky error word (a barrier that timed out); from
// bar[11 * 32]: one claim word per conv2 slab chunk (the conv1 "helpers", cnn_wgrad.hip).
#define DMLC_WBAR_WORDS (20 * 32)
struct DmlcWgradArgs {
  DmlcConv1WgradArgs w1;
  DmlcConv2WgradArgs w2;
  int apply;
  unsigned int* bar;
  int helpers;              // apply mode: idle conv1 blocks help reduce the conv2 slabs (B > 128)
  DmlcSgdArgs sgd;
  // apply mode with the fc chain (fc_in_launch): the conv1 blocks, whose conv1 work ends ~8 us before
  // the conv2 blocks', also run the fc weight-gradient tiles (dW1 / dW2 / dW3 + bias gradients,
  // fc_common.h) with every fc parameter's SGD in their epilogues (fc.fuse_sgd = 2): no fc SGD roles
  int fc_in_launch;
  DmlcFcArgs fc;
  int fc_done;              // apply mode: the fc chain already applied every fc SGD (fuse_sgd 2): no fc roles
};

hipError_t dmlc_conv1_fwd(const DmlcConv1FwdArgs* a, hipStream_t s);
hipError_t dmlc_conv2_fwd(const DmlcConv2FwdArgs* a, hipStream_t s);
// conv1 + pool1 + conv2 + pool2 of one image per workgroup in one launch (bf16; a1->amax must be null)
hipError_t dmlc_conv12_fwd(const DmlcConv1FwdArgs* a1, const DmlcConv2FwdArgs* a2, hipStream_t s);
// channel-split variants (cnn_split.hip): nsplit workgroups per image (B % 8 == 0), each owning
// 64 / nsplit output channels (conv1: nsplit 2 or 4; conv2 forward / input gradient: 2)
hipError_t dmlc_conv1_fwd_split(const DmlcConv1FwdArgs* a, int nsplit, hipStream_t s);
// conv1 + pool1 + conv2 + pool2 with two workgroups per image exchanging their pool1 halves in the
// launch (B <= 128; flags: 32 * 2B zeroed uints, err: the sticky error word)
hipError_t dmlc_conv12_fwd_split(const DmlcConv1FwdArgs* a1, const DmlcConv2FwdArgs* a2, unsigned* flags,
                                 unsigned* err, hipStream_t s);
hipError_t dmlc_conv2_fwd_split(const DmlcConv2FwdArgs* a, hipStream_t s);
hipError_t dmlc_conv2_dgrad_split(const DmlcConv2DgradArgs* a, hipStream_t s);
hipError_t dmlc_conv2_fwd_fp8(const DmlcConv2FwdFp8Args* a, hipStream_t s);
hipError_t dmlc_conv2_dgrad_fp8(const DmlcConv2DgradFp8Args* a, hipStream_t s);
hipError_t dmlc_fp8_roundtrip(const float* x, float* y, int n, float scale, hipStream_t s);
hipError_t dmlc_conv2_dgrad(const DmlcConv2DgradArgs* a, hipStream_t s);
// conv2 dgrad + the conv1 weight gradient of each image (one slab per image: w1->g1 == B, xraw set)
hipError_t dmlc_wgrad(const DmlcWgradArgs* a, hipStream_t s);
hipError_t dmlc_gemm_grouped(DmlcGemmGroup* g, hipStream_t s);
// dg: null, or the conv2 dgrad of the same batch, run in the chain's workgroups (dg->dp2 == a->dp2;
// a->sync >= 28 * 32 words)
hipError_t dmlc_fc_chain(const DmlcFcArgs* a, const DmlcConv2DgradArgs* dg, hipStream_t s);
hipError_t dmlc_head(const DmlcHeadArgs* a, hipStream_t s);
hipError_t dmlc_sgd(DmlcSgdArgs* a, hipStream_t s);

}  // extern "C"
