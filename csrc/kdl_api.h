// Host-callable entry points of the kubedl_amd HIP kernels (raw pointers,
// explicit stream).  Implemented in csrc/*.hip, bound in csrc/bindings.cpp.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kdl {

// ---- bn_act.hip (dtype codes: 0 = f32, 1 = bf16)
// ``ws`` is a per-layer fp32 workspace of bn_workspace_floats(C) elements,
// zero when first used; the kernels leave it zero again (self-cleaning).
int64_t bn_workspace_floats(int C);
// ``mbits`` (optional, bf16 with C % 8 == 0, relu + residual only): uint8 [M, C/8]
// ReLU mask written by the forward and read by the backward instead of y.
hipError_t bn_act_forward(const void* x, const void* res, void* y, uint8_t* mbits, const void* gamma,
                          const void* beta, float* rm, float* rv, float* save_mean,
                          float* save_invstd, float* ws, int64_t M, int C, int dtype, int pdtype,
                          bool relu, bool training, float momentum, float eps, hipStream_t s);
hipError_t bn_act_backward(const void* dy, const void* y, const uint8_t* mbits, const void* x,
                           const void* gamma,
                           const void* beta, const float* mean, const float* invstd, void* dx,
                           void* dres, void* dgamma, void* dbeta, float* ws, int64_t M, int C,
                           int dtype, int pdtype, bool relu, bool training, hipStream_t s);

// Stem BN + ReLU + max-pool(3, 2, 1), bf16 NHWC x [N, H, W, C], C % 8 == 0.
// y [N, PH, PW, C]; idx uint8 [N, PH, PW, C] = in-window argmax (kh*3 + kw).
hipError_t bn_pool_forward(const void* x, void* y, uint8_t* idx, const void* gamma, const void* beta,
                           float* rm, float* rv, float* save_mean, float* save_invstd, float* ws,
                           int N, int H, int W, int C, int pdtype, bool training, float momentum,
                           float eps, hipStream_t s,
                           bool gemm_stats = false, void* xam = nullptr);
hipError_t bn_pool_backward(const void* dyp, const uint8_t* idx, const void* x, const void* gamma,
                            const void* beta, const float* mean, const float* invstd, void* dx,
                            void* dgamma, void* dbeta, float* ws, int N, int H, int W, int C,
                            int pdtype, bool training, hipStream_t s,
                            bool with_dx = true);

// Staged BN entry points for the explicit ResNet engine (bf16 NHWC, C % 8 == 0).
// Forward: stats (or a conv1x1 STATS epilogue) -> finalize (shift = the K the sums
// were taken around: null = x[0, c]) -> apply (optional residual, or a second
// BN-normalised branch xd/wsd; optional packed mask).  Backward: mask_reduce (or a
// conv1x1 MASKX/RESBITS epilogue) -> finalize -> apply (g already masked;
// optional second branch).
hipError_t bn_stage_fwd_stats(const void* x, float* ws, int64_t M, int C, hipStream_t s);
hipError_t bn_stage_fwd_finalize(const void* x, const float* shift, float* ws, int64_t M, int C, const void* gamma,
                                 const void* beta, float* rm, float* rv, float* save_mean, float* save_invstd,
                                 int pdtype, bool training, float momentum, float eps, hipStream_t s);
const float* bn_stage_coef(const float* ws, int C);
hipError_t bn_stage_fwd_apply(const void* x, const float* ws, const void* res, const void* xd, const float* wsd,
                              void* y, uint8_t* mbits, int64_t M, int C, bool relu, hipStream_t s);
hipError_t bn_stage_bwd_mask_reduce(const void* dy, int dy_rows_per_img, float dy_scale, const uint8_t* mbits,
                                    const void* x, const float* mean, void* gout, float* ws, int64_t M, int C,
                                    const void* x2, const float* mean2, float* ws2, hipStream_t s);
// BN+ReLU backward with the ReLU mask recomputed from x (relu_mask_x) or no mask:
// reduce (sums only) -> finalize -> apply_maskx.
hipError_t bn_stage_bwd_reduce(const void* dy, const void* x, const void* gamma, const void* beta, const float* mean,
                               const float* invstd, float* ws, int64_t M, int C, bool relu_mask_x, int pdtype,
                               hipStream_t s);
hipError_t bn_stage_bwd_apply_maskx(const void* dy, const void* x, const void* gamma, const void* beta,
                                    const float* mean, const float* invstd, const float* ws, void* dx, int64_t M,
                                    int C, int pdtype, hipStream_t s);
hipError_t bn_stage_bwd_finalize(float* ws, int64_t M, int C, const void* gamma, const float* mean,
                                 const float* invstd, void* dgamma, void* dbeta, int pdtype, bool training,
                                 hipStream_t s);
hipError_t bn_stage_bwd_apply(const void* g, const void* x, const float* ws, void* dx, const void* xd,
                              const float* wsd, void* dxd, int64_t M, int C, hipStream_t s);

// ---- optim.hip
struct OptChunk {
  int64_t start;
  int32_t len;
  int32_t group;
};

struct OptHyper {
  float lr;
  float momentum;
  float dampening;
  float eps;
  float bc1;
  float bc2;
  float grad_scale;
  int nesterov;
  int first_step;
  int adam_w;
  float wd[4];
  float lr_scale[4];
};

hipError_t fused_sgd(const OptChunk* chunks, int nchunks, float* master, float* mom,
                     const void* grad, void* param, int gdtype, int pdtype, const OptHyper& h,
                     hipStream_t s);
hipError_t fused_adam(const OptChunk* chunks, int nchunks, float* master, float* m1, float* m2,
                      const void* grad, void* param, int gdtype, int pdtype, const OptHyper& h,
                      hipStream_t s);
hipError_t chunk_sumsq(const OptChunk* chunks, int nchunks, const void* x, int dtype, float scale,
                       float* out, hipStream_t s);
// ---- multi_tensor.hip
struct PackChunk {
  int32_t tensor;  // index into the per-step source pointer table
  int32_t len;     // elements
  int64_t src_off; // element offset inside the source tensor
  int64_t dst_off; // element offset inside the flat destination
};
// One 64x64 tile of a batched bf16 transpose dst[c * dst_ld + r] = src[r * src_ld + c]
// (r < rows, c < cols).
struct TransposeTile {
  const uint16_t* src;
  uint16_t* dst;
  int rows, cols;
  int r0, c0;
  int src_ld, dst_ld;
};
hipError_t transpose_tiles(const TransposeTile* tiles, int ntiles, hipStream_t s);
// source pointers as kernel arguments (pack_tensors ``args``): up to this many tensors
constexpr int kPackArgPtrs = 256;
struct PackPtrs {
  const void* p[kPackArgPtrs];
};
hipError_t pack_tensors(const PackChunk* chunks, int nchunks, const int64_t* src_ptrs, void* dst,
                        int dtype, float scale, hipStream_t s,
                        const PackPtrs* args = nullptr);

// ---- p2p.hip (two-phase all-reduce over IPC-mapped peer buffers)
constexpr int kP2PMaxRanks = 8;
constexpr int kP2PMaxBlocks = 128;
// Signal buffer per rank: uint32 [3 phases][kP2PMaxBlocks][kP2PMaxRanks].
constexpr int kP2PSignalWords = 3 * kP2PMaxBlocks * kP2PMaxRanks;
struct P2PArgs {
  void* buf[kP2PMaxRanks];      // bucket start in every rank's buffer (buf[rank] = own, local)
  uint32_t* sig[kP2PMaxRanks];  // every rank's signal buffer (peer-mapped)
  uint32_t* err;                // host-mapped error word: bit p = a phase-p wait timed out
  uint64_t timeout_ticks;       // per wait, in 100 MHz wall-clock ticks
  uint32_t units;               // 16-byte units in the bucket
  uint32_t epoch;               // call number (same sequence on every rank, starts at 1)
  float scale;                  // applied to the sum (1/world for an average)
  int rank, world;
};
int p2p_blocks(int64_t units, int world);
int p2p_oneshot_max_units();
// oneshot: whole bucket summed by every rank (units <= p2p_oneshot_max_units())
hipError_t p2p_allreduce(const P2PArgs& a, bool bf16, bool oneshot, hipStream_t s);

// ---- gbdt.hip (histogram GBDT for the XGBoostJob worker)
// one boosting round's gradient / hessian (obj 0 reg:squarederror, 1 binary:logistic,
// 2 multi:softprob; pred / g / h [n, K] fp32, y [n] fp32 labels / class ids)
hipError_t gbdt_grad_hess(const float* pred, const float* y, int64_t n, int K, int obj, float* g, float* h,
                          hipStream_t s);
hipError_t gbdt_hist_build(const uint8_t* bins, const float* grad, const float* hess, int64_t gh_stride,
                           const int32_t* rows, const int32_t* seg, int num_nodes, int max_rows_per_node,
                           int F, int B, float* hist, hipStream_t s);
hipError_t gbdt_split_find(const float* hist, int num_nodes, int F, int B, float lambda,
                           float min_child_weight, float* best_gain, int32_t* best_bin, float* best_gl,
                           float* best_hl, float* node_tot, hipStream_t s);
// device-resident growth (see gbdt.hip header)
// gh_max: {max |g|, max h} of the rows (gbdt_gh_absmax): the fixed-point scale
// of the quantised per-block sums
hipError_t gbdt_gh_absmax(const float* grad, const float* hess, int n, float* out, hipStream_t s);
// a tree's state reset (rows = iota, node_pos = 0, heap arrays -1 / 0, root bounds, root histogram)
hipError_t gbdt_tree_init(int32_t* rows, int32_t* node_pos, int N, int32_t* feat, int32_t* tbin, float* thr,
                          float* val, int heap, int32_t* exists0, int32_t* lo0, int32_t* hi0, float* root, int root_n,
                          hipStream_t s);
// node_of_row[rows[p]] = node_pos[p], then pred[r * ld + k] += val[node_of_row[r]]
hipError_t gbdt_leaf_add(float* pred, int ld, int k, const float* val, const int32_t* rows, const int32_t* node_pos,
                         int N, int32_t* node_of_row, hipStream_t s);
// out [4, heap] fp32 = (feat, tbin, thr, val)
hipError_t gbdt_heap_pack(const int32_t* feat, const int32_t* tbin, const float* thr, const float* val, int heap,
                          float* out, hipStream_t s);
// quantised histogram build: 0 = slot kernel (a wave = 64 / fp rows x fp features), 4 | 8 = row-per-lane
// kernel with that many rows in flight per lane (F % 4 == 0); -2 = KDL_TUNE gbdt_hist_rows
void set_gbdt_hist_rows(int u);
// row-per-lane build: 1 = g and h in one 64-bit LDS add, 0 = two 32-bit adds, -1 = KDL_TUNE gbdt_pack64
void set_gbdt_pack64(int p);
hipError_t gbdt_hist_wq(const uint8_t* bins, const float* grad, const float* hess, int64_t gh_stride,
                        const int32_t* rows, const int32_t* blo, const int32_t* bhi, int32_t* chunk_off, int nb,
                        int max_chunks, int rpb, int F, int B, const float* gh_max, float* hist, hipStream_t s);
hipError_t gbdt_decide(const float* gain, const int32_t* sbin, const float* tot, const float* cuts,
                       const int32_t* exists, int L, int F, int ncut, int h0, int can_split, float lambda,
                       float gamma, float lr, int32_t* t_feat, int32_t* t_bin, float* t_thr, float* t_val,
                       int32_t* split, int32_t* exists_next, hipStream_t s);
// node_pos: the heap node of the row at each POSITION (moved with the rows by gbdt_partition);
// feature_major: bins is the [F, N] copy (bins[f * n + row]), else [N, F]
hipError_t gbdt_route_flags(const uint8_t* bins, const int32_t* rows, const int32_t* node_pos,
                            const int32_t* split, const int32_t* t_feat, const int32_t* t_bin, int F, int n, int h0,
                            int L, int32_t* flag, hipStream_t s, bool feature_major = false);
// route + inclusive scan of the flags in one launch (single-pass, decoupled look-back): flag and
// sc as gbdt_route_flags + an inclusive scan.  status: gbdt_route_scan_tiles(n) zeroed words;
// ticket: one zeroed counter (re-armed by the kernel); epoch: 1, 2, ... per call on that status
// array (< 2^31); fault: counts look-backs that timed out (expected 0)
int gbdt_route_scan_tiles(int n);
hipError_t gbdt_route_scan(const uint8_t* bins, const int32_t* rows, const int32_t* node_pos, const int32_t* split,
                           const int32_t* t_feat, const int32_t* t_bin, int F, int n, int h0, int L, int32_t* flag,
                           int32_t* sc, unsigned long long* status, unsigned* ticket, uint32_t epoch, int* fault,
                           hipStream_t s);
hipError_t gbdt_partition(const int32_t* rows, const int32_t* node_pos, const int32_t* split, const int32_t* lo,
                          const int32_t* hi, const int32_t* flag, const int32_t* sc, int n, int h0, int L,
                          int32_t* rows_next, int32_t* node_pos_next, hipStream_t s);
// a level's routing + stable partition + child segments in three launches (route_count_kernel,
// level_plan_kernel, partition_tiles_kernel): the outputs of route_flags + scan + partition +
// children.  tincl: n ints (the tile-local scan); tile_cnt / tile_off: gbdt_level_tiles(n) ints;
// node_base / node_r: L ints
int gbdt_level_tiles(int n);
hipError_t gbdt_route_partition(const uint8_t* bins, bool feature_major, int F, const int32_t* rows,
                                const int32_t* node_pos, const int32_t* split, const int32_t* t_feat,
                                const int32_t* t_bin, const int32_t* lo, const int32_t* hi, int n, int h0, int L,
                                int32_t* flag, int32_t* tincl, int32_t* tile_cnt, int32_t* tile_off,
                                int32_t* node_base, int32_t* node_r, int32_t* rows_next, int32_t* node_pos_next,
                                int32_t* lo_next, int32_t* hi_next, float* cnt, int pick, int32_t* build_child,
                                int32_t* blo, int32_t* bhi, hipStream_t s);
hipError_t gbdt_children(const int32_t* split, const int32_t* lo, const int32_t* hi, const int32_t* sc, int L,
                         int32_t* lo_next, int32_t* hi_next, float* cnt, int pick, int32_t* build_child,
                         int32_t* blo, int32_t* bhi, hipStream_t s);
hipError_t gbdt_pick_small(const float* cnt, const int32_t* lo_next, const int32_t* hi_next, int L,
                           int32_t* build_child, int32_t* blo, int32_t* bhi, hipStream_t s);
hipError_t gbdt_subtract(const float* parent, float* built, const int32_t* split, const int32_t* build_child,
                         int L, int per_node, float* next, hipStream_t s);
hipError_t gbdt_quantise(const float* X, const float* cuts, int64_t n, int F, int ncut, int max_code, uint8_t* out,
                         hipStream_t s);
hipError_t gbdt_route_rows(const uint8_t* bins, const int32_t* rows, const int32_t* row_node,
                           const int32_t* split_feat, const int32_t* split_bin, int F, int n,
                           int32_t* go_right, hipStream_t s);

// ---- ctr.hip (XDLJob CTR model: MFMA GEMM, embeddings, sparse Adagrad)
// b_kn: B is [K][N] (C = A B), else [N][K] (C = A B^T)
hipError_t gemm_bias_act(const void* A, const void* B, const void* bias, bool bias_bf16, void* C, int M, int N, int K,
                         bool relu, bool b_kn, hipStream_t s);
void set_ctr_tile(int t);  // -1 by shape, 0/1/2: 128x128 / 128x64 / 64x64 (csrc/ctr.hip)
int ctr_tile_for(int M, int N);
// forward gemm_bias_act on the LDS-DMA igemm loop: 0 off, 1 by tile count, 2 every
// K % 64 / N % 64 shape; cfg -1 by shape (igemm tile configs 0-4)
void set_ctr_igemm(int mode, int cfg);
// the split reductions' hand-off: 1 = sc1 partials, no fences; 0 = fenced; -1 = KDL_TUNE ctr_handoff
void set_ctr_handoff(int sc1);
int ctr_igemm_cfg_for(int M, int N, int K);  // -1: the register-staged kernel
// part: relu_bwd_dbias_parts(M, N) x [N] fp32 scratch; cnt: (N + 255) / 256 counters,
// zero before the first call (the kernel re-arms them); db: [N] bf16 (db_bf16) or fp32
int relu_bwd_dbias_parts(int M, int N);
// C = (A W) masked by y > 0 (W [K, N]: the data gradient into the previous layer's ReLU output y),
// db = column sums of C (bf16, deterministic); part: gemm_dgrad_relu_tiles_m(M, N) x [N] fp32
// scratch; cnt: ceil(N / 64) zeroed ticket counters (re-armed by the kernel)
int gemm_dgrad_relu_tiles_m(int M, int N);
hipError_t gemm_dgrad_relu(const void* A, const void* B, const void* y, void* C, float* part, unsigned* cnt, void* db,
                           int M, int N, int K, hipStream_t s);
hipError_t relu_bwd_dbias(const void* dy, const void* y, void* dz, float* part, unsigned* cnt, void* db, bool db_bf16,
                          int M, int N, hipStream_t s);
// cnt: one ticket counter, zero before the first call (re-armed by the kernel);
// loss [1] fp32 = the mean loss; b: bf16 (b_bf16) or fp32 [1]
int head_bce_fwd_blocks(int M);  // = the loss-partial count
hipError_t head_bce_fwd(const void* x, const void* w, const void* b, bool b_bf16, const float* y, int M, int K,
                        float* logit, float* dlogit, float* loss_part, unsigned* cnt, float* loss, hipStream_t s);
int head_bce_bwd_blocks(int M);
// dw / db (bf16 [K] / [1], optional): the partials summed in block order by the last block
hipError_t head_bce_bwd(const void* x, const void* w, const float* dlogit, float scale, const float* gscale, int M,
                        int K, void* dx, float* dw_part, float* db_part, unsigned* cnt, void* dw, void* db,
                        hipStream_t s, float* dbx_part = nullptr, void* dbx = nullptr);
// dbx (bf16 [K], needs dw and dbx_part [blocks][K]): x is a ReLU output -- dx is masked by x > 0
// and dbx = its column sums (the bias gradient of the layer that produced x)
// out[b, col0 + f*D : +D] = bf16(table[uniq[inv[b*F + f]]]) (fp32 table, bf16 out)
hipError_t embed_gather_cast(const void* table, bool table_bf16, const int64_t* uniq, const int64_t* inv, int n,
                             int F, int D, void* out, int ld_out, int col0, hipStream_t s,
                             const float* dense = nullptr, int nd = 0, int tail = 0);
hipError_t embed_gather(const void* table, int dtype, const int64_t* idx, int n, int F, int D, void* out, int ld_out,
                        int col0, hipStream_t s);
// ucount (optional): the live segment count on the device; U is then a capacity
hipError_t segment_reduce(const void* rows, int dtype, int F, int ld, int col0, const int64_t* order,
                          const int64_t* seg, int U, int D, float* out, hipStream_t s, const int* ucount,
                          int64_t nrows,  // nrows = order's length (B * F)
                          const int64_t* out_row = nullptr, int64_t out_lim = 0);  // out row of segment u (< out_lim)
// segment_reduce + a one-row-per-segment segment_adagrad in one launch: segment
// u's sum updates table/accum row rows_local[u] (rows outside [0, nrows) skipped)
hipError_t segment_reduce_adagrad(const void* rows, int dtype, int F, int ld, int col0, const int64_t* order,
                                  const int64_t* seg, int U, int D, const int* ucount, int64_t nrows_in,
                                  const int64_t* rows_local, int64_t nrows, float* table, float* accum, float lr,
                                  float eps, float scale, hipStream_t s);
// Fixed-capacity embedding exchange (models/ctr.py _pull_fixed / _push_fixed):
// route n unique ids (first *count live) to W destination blocks of cap + 1
// slots (send [W * (cap + 1)]: ids, -1 padding, header = the largest fill) and
// rslot [n] (d * cap + pos, W * cap = dump); cnt: a2a_route_blocks(n) * W ints.
int a2a_max_world();
int a2a_route_blocks(int n);
hipError_t a2a_route(const int64_t* uniq, const int* count, int n, const int64_t* owner_rank, int n_own, int W,
                     int cap, int* cnt, int64_t* send, int64_t* rslot, hipStream_t s);
// owner side: rows [n, D] = table[req / n_own] (zero for req < 0; fp32 or bf16),
// local [n] = req / n_own or -2 - r
// slotmap != nullptr: also stamp slotmap[local * W + slot / cap] = (call << 32) | slot
// (the owner update's stamps, a2a_owner_update(..., stamped = true); n = W * cap)
hipError_t a2a_serve(const float* table, const int64_t* req, int n, int n_own, int D, void* rows, bool rows_bf16,
                     int64_t* local, hipStream_t s, int64_t* slotmap = nullptr, int64_t call = 0, int cap = 0,
                     int W = 0, int64_t nrows = 0);
// owner update of a fixed exchange without de-duplication: grads [S = W * cap, D]
// fp32 with local rows local [S] (< 0 padding); slotmap [nrows * W] int64
// persistent (zero initially), call = 1, 2, ... (< 2^31) one per call
hipError_t a2a_owner_update(const float* grads, const int64_t* local, int S, int cap, int W, int D, int64_t nrows,
                            int64_t* slotmap, int64_t call, float* table, float* accum, float lr, float eps,
                            float scale, hipStream_t s, bool stamped = false);  // stamped: by a2a_serve
// rows_local outside [0, nrows) are skipped (exchange padding sentinels)
hipError_t segment_adagrad(const float* grads, const int64_t* order, const int64_t* seg, const int64_t* rows_local,
                           int U, int D, int64_t nrows, float* table, float* accum, float lr, float eps, float scale,
                           hipStream_t s, const int* ucount = nullptr);
// Sync-free de-duplication of n int64 ids (csrc/ctr.hip): uniq [n] (first *count
// valid, the rest padded with uniq[0]), inv [n], count [1] and the segment sizes
// [n + 1] on the device.  keys: T = dedup_table_slots(n) int64 slots, all -1
// initially (the call leaves them -1 again); slot_of [n], slot_uid [T], bsum [T / 1024].
int dedup_table_slots(int n);
hipError_t dedup_ids(const int64_t* ids, int n, void* keys, int T, int* slot_of, int* slot_uid, int* bsum,
                     int64_t* uniq, int64_t* inv, int* count, int* sizes, hipStream_t s);
// CSR of the inverse map: seg [n + 1] (exclusive scan of sizes), order [n] =
// positions grouped by unique id, ascending within each group (deterministic sums).
// bsum: csr_bsum_slots(n) ints.  sizes and cursor are clobbered (scratch of the
// long-segment sort).
int csr_bsum_slots(int n);
hipError_t csr_from_inverse(const int64_t* inv, int n, int* sizes, const int* count, int* bsum, int* cursor,
                            int64_t* seg, int64_t* order, hipStream_t s);


// ---- conv1x1.hip (ResNet 1x1 convs as MFMA GEMMs with fused BN prologue/epilogues)
// epi: 0 plain, 1 BN-forward stats, 2 ReLU-mask-from-x + BN-backward sums,
//      3 residual add + packed-bit mask + BN-backward sums (+ second BN), 4 residual add,
//      5 BN apply + residual + ReLU + packed mask out (ecoef = [2N] scale | shift).
// epi 1 with C == null: statistics only, nothing stored.
struct Conv1x1Args {
  const void* A;        // bf16 [rows, K]
  const void* B;        // bf16 [N, K]
  void* C;              // bf16 [M, N]
  int M, N, K;
  int Hout, Wout, Hin, Win, stride;  // stride > 1: A rows are gathered (strided 1x1 conv)
  const float* pro_coef;             // [2K] scale | shift -> A = relu(A*scale + shift); null = none
  int epi;
  const float* shift;                // epi 1: [N]
  float* acc;                        // epi 1-3: BN workspace replicas [32][2N]
  const void* ex;                    // epi 2-3: BN input [M, N]
  const float* emean;                // epi 2-3: [N]
  const float* ecoef;                // epi 2: [2N]
  const void* eres;                  // epi 3-4: d(identity)
  int res_stride, res_H, res_W;      // eres sampled at stride res_stride of the (res_H, res_W) grid
  const uint8_t* ebits;              // epi 3: [M, N/8]
  const void* ex2;                   // epi 3: optional second BN input
  const float* emean2;
  float* acc2;
  int ksize;                         // 1 (or 0): 1x1 conv / GEMM; 3: 3x3 pad-1 implicit GEMM (K = 9 * Cin)
  int Cin;                           // ksize 3: input channels (the A row width)
  float* fin_ws;                     // epi 1-3: finalize the BN of this workspace in the GEMM (bn_fin.h)
  float* fin_ws2;                    // epi 3: and the downsample BN's
  float fin_M;                       // their element count
  // BN-backward-apply prologue of A (dense 1x1 dgrad): A' = k A + c1 bx + c0,
  // bit-identical to bn_stage_bwd_apply's output; aout (optional) receives A'
  const void* bx;                    // that BN's input [M, K]
  const float* bcoef;                // [3K] its backward coefficients (ws_bcoef)
  const float* bcoef2;               // bres 2: the residual BN's [2K] scale | shift (no concatenated copy)
  void* aout;                        // [M, K]
  // bres = 1: the prologue is the closing BN + residual + ReLU of the previous
  // block, relu(A * bcoef[k] + bcoef[K + k] + bx), written through to aout
  // with its packed ReLU mask in obits [M, K / 8] (forward conv1, STATS)
  int bres;
  uint8_t* obits;                    // bres: the written-through block output's ReLU mask [M, K/8]
};
hipError_t conv1x1_gemm(const Conv1x1Args& a, hipStream_t s);
// Data gradient of a 3x3 / pad 1 / stride 2 conv as four sub-pixel class GEMMs
// on the LDS-DMA core (one launch): A = dy [Nb, Hin, Win, Cin], B = the weights
// regrouped class-major [N][9 Cin] (conv3x3_s2_dgrad_weights), C = dx
// [Nb, Hout, Wout, N] with Hout = 2 Hin or 2 Hin - 1 (an odd conv input: the last
// sub-pixel row is masked), likewise Wout; M = Nb * Hin * Win; epi PLAIN or MASKX
// (ex / emean / ecoef / acc as conv1x1_gemm, indexed by dx rows).
hipError_t conv3x3_dgrad_s2(const Conv1x1Args& a, hipStream_t s);
// ResNet stem conv (csrc/stem.hip): x [Nb, 224, 224, 3] NHWC bf16, wp = the
// weights as [64][224] bf16 (k = r * 32 + s * 4 + c, zero for s = 7 / c = 3),
// y [Nb, 112, 112, 64] NHWC; acc != null: BN statistics around shift into the
// forward replicas (STATS epilogue), else a plain store.
// raw_w: wp is the nn.Conv2d weight [64][3][7][7] itself (reordered while the
// kernel stages it), else [64][224] in stem_weights' K order.
// x [Nb, H, W, 3] NHWC (any H, W: 2-row x 112-column tiles, masked edges),
// y [Nb, OH, OW, 64], OH = (H - 1) / 2 + 1.
hipError_t stem7x7_fwd(const void* x, const void* wp, void* y, int Nb, int H, int W, const float* shift, float* acc,
                       hipStream_t s, bool raw_w = false);
// stem weight gradient: dy [Nb, OH, OW, 64], x [Nb, H, W, 3] (NHWC bf16)
// -> dW [64][224] bf16 in stem_weights' K order; dw32 = stem7x7_wgrad_slabs(Nb, H, W)
// x [64][224] fp32 slabs (no initialisation needed)
int stem7x7_wgrad_slabs(int Nb, int H = 224, int W = 224);
// raw_out: dW is written as the nn.Conv2d gradient [64][3][7][7] instead.
hipError_t stem7x7_wgrad(const void* dy, const void* x, float* dw32, void* dW, int Nb, int H, int W, hipStream_t s,
                         bool raw_out = false);
// the same with the stem BN + ReLU + max-pool backward folded in (224 x 224 only): dy is built
// per tile from c0 [Nb, 112, 112, 64], the pooled gradient dp [Nb, 56, 56, 64],
// its argmax bytes idx and coef5 = [5][64] (forward scale | shift, backward
// k | c1 | c0 of the BN workspace, after bn_pool_backward(with_dx = false))
hipError_t stem7x7_wgrad_bn(const void* c0, const void* dp, const uint8_t* idx, const float* coef5, const void* x,
                            float* dw32, void* dW, int Nb, hipStream_t s, bool raw_out = false);
// Classifier head (csrc/head.hip): x [Nb, HW, C] NHWC bf16 (last block output),
// fc weight w [L][C] bf16, bias b [L] bf16 (optional), labels y [Nb] int64.
// Forward: feat [Nb][C] bf16 (mean pool), part1 [s1][Nb][L] fp32 (split-K fc
// partials), lrow [Nb] per-image loss, dl [Nb][Lp] / dlT [L][Nb] bf16 dlogits
// (mean reduction).  Backward: part2 [s2][Nb][C] fp32, dfeat [Nb][C] bf16,
// dW [L][C] / db [L] bf16, loss [1] fp32 (mean).  s1 / s2 from head_splits.
void head_splits(int Nb, int C, int L, int* s1, int* s2);
int head_lpad(int L);  // dl's row pitch: L rounded up to 8
hipError_t head_forward(const void* x, int Nb, int HW, int C, const void* w, const void* b, int L, const int64_t* y,
                        void* feat, float* part1, float* lrow, void* dl, void* dlT, hipStream_t s);
hipError_t head_backward(const void* feat, const void* w, const void* dl, const void* dlT, int Nb, int C, int L,
                         float* part2, void* dfeat, void* dW, void* db, const float* lrow, float* loss,
                         hipStream_t s);
// fixed-order sum of nsplit fp32 [nk] slabs into bf16 (scaled), csrc/conv1x1.hip;
// layout 1: the stem's [64][224] K order written out as [64][3][7][7]
// Gram fold of a BN-backward weight gradient (csrc/conv1x1.hip): Q = a^T a and
// s = 1^T a of a = relu(X * scale + shift) (pro = [scale | shift], X [M, K] bf16)
// into ws[0 : K * K + K] (fp32; ws holds conv1x1_gram_splits(M, K) * (K * K + K)
// floats), and dW = diag(k) Gm + diag(c1) W Q + c0 s^T -> bf16 out [N, K]
// (bcoef = [k | c1 | c0], Gm = g^T a fp32 [N, K], W the conv weight [N, K] bf16)
int conv1x1_gram_splits(int M, int K);
hipError_t conv1x1_gram(const void* X, const float* pro, float* ws, int M, int K, hipStream_t s);
hipError_t gram_fold(const float* Gm, const float* QS, const void* W, const float* bcoef, int N, int K, void* out,
                     hipStream_t s);
hipError_t wgrad_slab_reduce(float* dw32, int64_t nk, int nsplit, float scale, void* dW, hipStream_t s,
                             int layout = 0);
void set_stem_drop(int bits);  // timing-only: skip the stem's MFMAs (1), epilogue (2), input staging (4)
// solo: nothing else shares the GPU (no weight-gradient side stream): more blocks per tile
int conv1x1_wgrad_splits(int M, int N, int K, bool solo = false);
// 256 x 256 weight-gradient tiles: 0 off, 1 3x3 only (default), 2 3x3 + 1x1 (ignored under KDL_TUNE wgrad_big)
void set_wgrad_big(int mode);
// dW = scale * sum_m G[m, :]^T pro(A)[m, :].  dw32 is the split-M slab workspace
// (conv1x1_wgrad_splits(M, N, K) x [N, K] fp32, no initialisation needed); the
// result goes to dW (bf16) if given, else as fp32 into the first [N, K] of dw32.
// gx / gcoef (optional): G is replaced by the BN-backward apply k G + c1 gx + c0
// (gcoef = [3N] k | c1 | c0), computed while staging it (LDS-DMA kernel only).
hipError_t conv1x1_wgrad(const void* G, const void* A, const float* pro_coef, float* dw32, void* dW, float scale,
                         int M, int N, int K, int Hout, int Wout, int Hin, int Win, int stride, hipStream_t s,
                         const void* gx = nullptr, const float* gcoef = nullptr, bool solo = false);
// 3x3 / pad 1: dW[Cout][3][3][Cin] = sum_m G[m, :]^T pro(A)_tap(m); dw32 holds
// conv3x3_wgrad_slabs(...) x [Cout, 9 Cin] fp32 (dw32_floats: its size; a smaller
// workspace of conv1x1_wgrad_splits(M, Cout, 9 Cin) slabs keeps the implicit GEMM).
int conv3x3_wgrad_slabs(int Nb, int Hin, int Win, int Cin, int Cout, int stride);
hipError_t conv3x3_wgrad(const void* G, const void* A, const float* pro_coef, float* dw32, int64_t dw32_floats,
                         void* dW, float scale, int Nb, int Hin, int Win, int Cin, int Cout, int stride,
                         hipStream_t s);

hipError_t cast_copy(const void* src, int sdtype, void* dst, int ddtype, int64_t n, hipStream_t s);

// ---- streams.hip
// dedicated = the stream gets a hardware queue of its own (full CU mask).
hipError_t make_stream(bool dedicated, int priority, hipStream_t* out, int cus = 0);
// one wave busy-waiting ``microseconds`` (queue-concurrency probe)
hipError_t spin(hipStream_t s, double microseconds);

// conv GEMM main-loop selection (-1 by shape, 0 register-staged, 1 LDS-DMA)
int gemm_core_mode();
void set_gemm_core_mode(int m);
// force an LDS-DMA tile config (-1 = by shape; csrc/igemm.hip igemm_pick)
void set_igemm_cfg(int cfg);
void set_halo3x3(int on);  // 0: every 3x3 on the implicit GEMM (A/B switch; KDL_TUNE halo=0)

}  // namespace kdl
