// Native driver of the device-resident GBDT level pipeline (csrc/gbdt.hip).
//
// ``GbdtGrower`` owns every per-tree workspace of one training job (row order,
// per-row heap node, per-level segments, histograms, the tree's heap arrays)
// and enqueues the fixed kernel sequence of each level on the current HIP
// stream.  Nothing in a tree reads device memory from the host: split
// decisions, child segments and the smaller-child choice stay on the GPU, so a
// whole tree is a stream of ~10 launches per level.
//
// Single rank: ``grow_local`` runs the whole tree in C++.  Several ranks: the
// Python caller interleaves the two collectives of each level (child counts,
// built histograms) between ``level_a`` / ``level_b`` / ``level_c``, which is
// exactly where the reference's rabit all-reduce sits in XGBoost's hist
// updater.
#include <cstdlib>
#include <algorithm>
#include <torch/extension.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "kdl_api.h"
#include "tune.h"

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

void ck(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "kubedl_amd: ", what, " failed: ", hipGetErrorString(e));
}

int32_t* ip(const at::Tensor& t) { return t.data_ptr<int32_t>(); }
float* fp(const at::Tensor& t) { return t.data_ptr<float>(); }

class GbdtGrower {
 public:
  GbdtGrower(const at::Tensor& bins, const at::Tensor& cuts, int64_t num_bins, int64_t max_depth, double lambda,
             double gamma, double lr, double min_child_weight)
      : bins_(bins), cuts_(cuts.to(at::kFloat).contiguous()) {
    TORCH_CHECK(bins.is_cuda() && bins.scalar_type() == at::kByte && bins.dim() == 2 && bins.is_contiguous(),
                "GbdtGrower: bins must be a contiguous uint8 [N, F] GPU tensor");
    TORCH_CHECK(num_bins >= 2 && num_bins <= 256, "GbdtGrower: 2 <= num_bins <= 256");
    TORCH_CHECK(max_depth >= 0 && max_depth <= 10, "GbdtGrower: max_depth <= 10");
    N_ = static_cast<int>(bins.size(0));
    F_ = static_cast<int>(bins.size(1));
    B_ = static_cast<int>(num_bins);
    D_ = static_cast<int>(max_depth);
    TORCH_CHECK(cuts_.dim() == 2 && cuts_.size(0) == F_ && cuts_.device() == bins.device(),
                "GbdtGrower: cuts [F, ncut] on the bins' device");
    TORCH_CHECK((static_cast<int64_t>(F_) * B_) % 2 == 0, "GbdtGrower: F * num_bins must be even (float4 hist)");
    TORCH_CHECK(static_cast<int64_t>(N_) * F_ < (1LL << 31), "GbdtGrower: N * F must fit in int32");
    ncut_ = static_cast<int>(cuts_.size(1));
    lam_ = static_cast<float>(lambda);
    gamma_ = static_cast<float>(gamma);
    lr_ = static_cast<float>(lr);
    mcw_ = static_cast<float>(min_child_weight);
    // rows per histogram chunk (also the quantisation's per-block row bound,
    // csrc/gbdt.hip): the smallest power of two giving <= 512 chunks over the
    // root (two resident blocks per CU), 256..4096.  Every chunk's block ends in
    // a 57 KB flush of agent-scope float atomics (2M x 28), paid per block: with
    // the row-per-lane build the flush, not the LDS adds, bounds small chunks --
    // 2M x 28, depth 6: 1024 / 2048 / 4096 / 8192 rows per chunk 578-793 /
    // 941-946 / 1005-1007 / 934-939 boosting rounds/s (profiles/r06_gbdt_rpb.txt;
    // the round-2 float-atomic build preferred 1024).  KDL_TUNE gbdt_rpb overrides.
    const int64_t target = std::max(0, kdl::tune_int("gbdt_rpb", 0));
    rpb_ = 256;
    if (target > 0) {
      rpb_ = static_cast<int>(target);
    } else {
      while (rpb_ < 4096 && static_cast<int64_t>(rpb_) * 512 < N_) rpb_ *= 2;
    }

    const c10::hip::HIPGuardMasqueradingAsCUDA guard(bins.device());
    auto io = bins.options().dtype(at::kInt);
    auto fo = bins.options().dtype(at::kFloat);
    const int64_t maxL = 1LL << D_, heap = (1LL << (D_ + 1)) - 1;
    iota_ = at::arange(N_, io);
    rows_ = at::empty({N_}, io);
    rows_next_ = at::empty({N_}, io);
    node_of_row_ = at::zeros({N_}, io);
    node_pos_ = at::empty({N_}, io);
    node_pos_next_ = at::empty({N_}, io);
    // feature-major copy of the bin codes for the routing passes (route_flags_kernel): N x F bytes
    bins_t_ = bins_.t().contiguous();
    flag_ = at::empty({N_}, io);
    sc_ = at::empty({N_}, io);
    // fused route + scan (csrc/gbdt.hip route_scan_kernel): look-back words, tile ticket, fault count
    scan_status_ = at::zeros({std::max(1, kdl::gbdt_route_scan_tiles(N_))}, io.dtype(at::kLong));
    scan_ticket_ = at::zeros({1}, io);
    scan_fault_ = at::zeros({1}, io);
    // the three-launch level (gbdt_route_partition): tile counts / offsets (sc_ holds the
    // tile-local scan there), node bases and right counts
    tile_cnt_ = at::empty({std::max(1, kdl::gbdt_level_tiles(N_))}, io);
    tile_off_ = at::empty({std::max(1, kdl::gbdt_level_tiles(N_))}, io);
    node_base_ = at::empty({maxL}, io);
    node_r_ = at::empty({maxL}, io);
    for (int d = 0; d <= D_; ++d) {
      lo_.push_back(at::zeros({1LL << d}, io));
      hi_.push_back(at::zeros({1LL << d}, io));
      exists_.push_back(at::zeros({1LL << d}, io));
    }
    split_ = at::zeros({maxL}, io);
    gain_ = at::empty({maxL, F_}, fo);
    sbin_ = at::empty({maxL, F_}, io);
    gl_ = at::empty({maxL, F_}, fo);
    hl_ = at::empty({maxL, F_}, fo);
    tot_ = at::empty({maxL, 2}, fo);
    feat_ = at::empty({heap}, io);
    tbin_ = at::empty({heap}, io);
    thr_ = at::empty({heap}, fo);
    val_ = at::empty({heap}, fo);
    per_node_ = static_cast<int64_t>(F_) * B_ * 2;
    hist_cur_ = at::empty({maxL, F_, B_, 2}, fo);
    hist_next_ = at::empty({maxL, F_, B_, 2}, fo);
    // zeroed here and by every level's subtract once read (no fill per level)
    built_ = at::zeros({std::max<int64_t>(maxL / 2, 1), F_, B_, 2}, fo);
    cnt_ = at::zeros({maxL}, fo);
    build_child_ = at::zeros({std::max<int64_t>(maxL / 2, 1)}, io);
    blo_ = at::zeros({std::max<int64_t>(maxL / 2, 1)}, io);
    bhi_ = at::zeros({std::max<int64_t>(maxL / 2, 1)}, io);
    chunk_off_ = at::zeros({std::max<int64_t>(maxL / 2, 1) + 1}, io);
    root_lo_hi_ = at::tensor({0, N_}, io.device(at::kCPU)).to(bins.device());
    gh_max_ = at::zeros({2}, fo);
  }

  // Reset the per-tree state and build the root histogram (returned: the
  // caller all-reduces it in place when there are several ranks).
  at::Tensor begin_tree(const at::Tensor& grad, const at::Tensor& hess) {
    TORCH_CHECK(grad.is_cuda() && grad.scalar_type() == at::kFloat && grad.is_contiguous() && grad.numel() == N_,
                "GbdtGrower: grad must be contiguous fp32 [N]");
    TORCH_CHECK(hess.is_cuda() && hess.scalar_type() == at::kFloat && hess.is_contiguous() && hess.numel() == N_,
                "GbdtGrower: hess must be contiguous fp32 [N]");
    const c10::hip::HIPGuardMasqueradingAsCUDA guard(bins_.device());
    grad_ = grad;
    hess_ = hess;
    auto root = hist_cur_.narrow(0, 0, 1);
    ck(kdl::gbdt_tree_init(ip(rows_), ip(node_pos_), N_, ip(feat_), ip(tbin_), fp(thr_), fp(val_),
                           static_cast<int>(feat_.numel()), ip(exists_[0]), ip(lo_[0]), ip(hi_[0]), fp(root),
                           static_cast<int>(root.numel()), stream()),
       "gbdt_tree_init");
    // the tree's fixed-point scale of the quantised histogram sums (csrc/gbdt.hip)
    ck(kdl::gbdt_gh_absmax(fp(grad_), fp(hess_), N_, fp(gh_max_), stream()), "gbdt_gh_absmax");
    const int max_chunks = (N_ + rpb_ - 1) / rpb_ + 1;
    ck(kdl::gbdt_hist_wq(bins_.data_ptr<uint8_t>(), fp(grad_), fp(hess_), 1, ip(rows_), ip(root_lo_hi_),
                         ip(root_lo_hi_) + 1, ip(chunk_off_), 1, max_chunks, rpb_, F_, B_, fp(gh_max_), fp(root),
                         stream()),
       "gbdt_hist_wq(root)");
    builds_ += 1;
    return root;
  }

  // Level d: split search + decisions; below max depth also route, partition
  // and child segments.  Returns the child row counts [2L] (all-reduce them
  // and call ``level_b(d, true)`` when ranks > 1), or an empty tensor at the
  // last level.
  at::Tensor level_a(int64_t d, bool pick) {
    const c10::hip::HIPGuardMasqueradingAsCUDA guard(bins_.device());
    const int L = 1 << d, h0 = L - 1;
    const bool last = d >= D_;
    ck(kdl::gbdt_split_find(fp(hist_cur_), L, F_, B_, lam_, mcw_, fp(gain_), ip(sbin_), fp(gl_), fp(hl_), fp(tot_),
                            stream()),
       "gbdt_split_find");
    ck(kdl::gbdt_decide(fp(gain_), ip(sbin_), fp(tot_), fp(cuts_), ip(exists_[d]), L, F_, ncut_, h0, last ? 0 : 1,
                        lam_, gamma_, lr_, ip(feat_), ip(tbin_), fp(thr_), fp(val_), ip(split_),
                        last ? nullptr : ip(exists_[d + 1]), stream()),
       "gbdt_decide");
    if (last) return at::Tensor();
    if (route_plan_on()) {
      // route + per-tile / per-node counts, one-block plan (tile offsets, node bases, child
      // segments), partition: three launches instead of route + scan (2) + partition + children
      ck(kdl::gbdt_route_partition(bins_t_.data_ptr<uint8_t>(), true, F_, ip(rows_), ip(node_pos_), ip(split_),
                                   ip(feat_), ip(tbin_), ip(lo_[d]), ip(hi_[d]), N_, h0, L, ip(flag_), ip(sc_),
                                   ip(tile_cnt_), ip(tile_off_), ip(node_base_), ip(node_r_), ip(rows_next_),
                                   ip(node_pos_next_), ip(lo_[d + 1]), ip(hi_[d + 1]), fp(cnt_), pick ? 1 : 0,
                                   ip(build_child_), ip(blo_), ip(bhi_), stream()),
         "gbdt_route_partition");
      std::swap(rows_, rows_next_);
      std::swap(node_pos_, node_pos_next_);
      return cnt_.narrow(0, 0, 2 * L);
    }
    if (route_scan_on()) {
      if (++scan_epoch_ >= (1u << 31)) {  // epochs wrapped: start the words over
        scan_status_.zero_();
        scan_epoch_ = 1;
      }
      ck(kdl::gbdt_route_scan(bins_.data_ptr<uint8_t>(), ip(rows_), ip(node_pos_), ip(split_), ip(feat_), ip(tbin_),
                              F_, N_, h0, L, ip(flag_), ip(sc_),
                              reinterpret_cast<unsigned long long*>(scan_status_.data_ptr<int64_t>()),
                              reinterpret_cast<unsigned*>(ip(scan_ticket_)), scan_epoch_, ip(scan_fault_), stream()),
         "gbdt_route_scan");
    } else {
      ck(kdl::gbdt_route_flags(bins_t_.data_ptr<uint8_t>(), ip(rows_), ip(node_pos_), ip(split_), ip(feat_),
                               ip(tbin_), F_, N_, h0, L, ip(flag_), stream(), true),
         "gbdt_route_flags");
      at::cumsum_out(sc_, flag_, 0, at::kInt);
    }
    ck(kdl::gbdt_partition(ip(rows_), ip(node_pos_), ip(split_), ip(lo_[d]), ip(hi_[d]), ip(flag_), ip(sc_), N_,
                           h0, L, ip(rows_next_), ip(node_pos_next_), stream()),
       "gbdt_partition");
    std::swap(rows_, rows_next_);
    std::swap(node_pos_, node_pos_next_);
    ck(kdl::gbdt_children(ip(split_), ip(lo_[d]), ip(hi_[d]), ip(sc_), L, ip(lo_[d + 1]), ip(hi_[d + 1]), fp(cnt_),
                          pick ? 1 : 0, ip(build_child_), ip(blo_), ip(bhi_), stream()),
       "gbdt_children");
    return cnt_.narrow(0, 0, 2 * L);
  }

  // Build the histogram of each split node's smaller child (returned [L, F,
  // B, 2]: all-reduce it when ranks > 1).  ``pick``: choose the smaller child
  // from the (all-reduced) counts now.
  at::Tensor level_b(int64_t d, bool pick) {
    const c10::hip::HIPGuardMasqueradingAsCUDA guard(bins_.device());
    const int L = 1 << d;
    if (pick)
      ck(kdl::gbdt_pick_small(fp(cnt_), ip(lo_[d + 1]), ip(hi_[d + 1]), L, ip(build_child_), ip(blo_), ip(bhi_),
                              stream()),
         "gbdt_pick_small");
    auto built = built_.narrow(0, 0, L);  // zero: level_c's subtract cleared what the last build wrote
    const int max_chunks = (N_ + rpb_ - 1) / rpb_ + L;
    ck(kdl::gbdt_hist_wq(bins_.data_ptr<uint8_t>(), fp(grad_), fp(hess_), 1, ip(rows_), ip(blo_), ip(bhi_),
                         ip(chunk_off_), L, max_chunks, rpb_, F_, B_, fp(gh_max_), fp(built), stream()),
       "gbdt_hist_wq");
    builds_ += L;
    return built;
  }

  // Children's histograms: built one copied, sibling = parent - built.
  void level_c(int64_t d) {
    const c10::hip::HIPGuardMasqueradingAsCUDA guard(bins_.device());
    const int L = 1 << d;
    ck(kdl::gbdt_subtract(fp(hist_cur_), fp(built_), ip(split_), ip(build_child_), L, static_cast<int>(per_node_),
                          fp(hist_next_), stream()),
       "gbdt_subtract");
    std::swap(hist_cur_, hist_next_);
    subtracted_ += L;
  }

  // Whole tree on one rank.
  void grow_local(const at::Tensor& grad, const at::Tensor& hess) {
    begin_tree(grad, hess);
    for (int d = 0; d <= D_; ++d) {
      level_a(d, true);
      if (d < D_) {
        level_b(d, false);
        level_c(d);
      }
    }
  }

  // the row-indexed leaf of every row, as of the last add_leaf
  at::Tensor node_of_row() const { return node_of_row_; }
  // pred[:, k] += leaf value of each row (pred [N, K] fp32 contiguous)
  void add_leaf(at::Tensor pred, int64_t k) {
    TORCH_CHECK(pred.is_cuda() && pred.scalar_type() == at::kFloat && pred.is_contiguous() && pred.dim() == 2 &&
                    pred.size(0) == N_ && k >= 0 && k < pred.size(1),
                "GbdtGrower.add_leaf: pred [N, K] fp32 contiguous, 0 <= k < K");
    const c10::hip::HIPGuardMasqueradingAsCUDA guard(bins_.device());
    ck(kdl::gbdt_leaf_add(fp(pred), static_cast<int>(pred.size(1)), static_cast<int>(k), fp(val_), ip(rows_),
                          ip(node_pos_), N_, ip(node_of_row_), stream()),
       "gbdt_leaf_add");
  }
  // the current tree's heap arrays as one [4, heap] fp32 tensor (feature, split bin, threshold, value)
  at::Tensor heap_packed() const {
    const c10::hip::HIPGuardMasqueradingAsCUDA guard(bins_.device());
    const int64_t heap = feat_.numel();
    auto out = at::empty({4, heap}, thr_.options());
    ck(kdl::gbdt_heap_pack(ip(feat_), ip(tbin_), fp(thr_), fp(val_), static_cast<int>(heap), fp(out), stream()),
       "gbdt_heap_pack");
    return out;
  }
  // (feature, split_bin, threshold, value) heap arrays of the current tree
  std::vector<at::Tensor> tree() const { return {feat_, tbin_, thr_, val_}; }
  std::vector<int64_t> stats() const { return {builds_, subtracted_}; }
  // look-backs of the fused route + scan that timed out (syncs; expected 0)
  int64_t scan_faults() const { return scan_fault_.item<int>(); }
  int64_t rows_per_chunk() const { return rpb_; }

 private:
  at::Tensor bins_, bins_t_, cuts_, grad_, hess_;
  int N_ = 0, F_ = 0, B_ = 0, D_ = 0, ncut_ = 0, rpb_ = 256;
  float lam_ = 1.f, gamma_ = 0.f, lr_ = 0.3f, mcw_ = 1.f;
  int64_t per_node_ = 0, builds_ = 0, subtracted_ = 0;
  at::Tensor iota_, rows_, rows_next_, node_of_row_, node_pos_, node_pos_next_, flag_, sc_, root_lo_hi_;
  std::vector<at::Tensor> lo_, hi_, exists_;
  at::Tensor split_, gain_, sbin_, gl_, hl_, tot_, feat_, tbin_, thr_, val_;
  at::Tensor hist_cur_, hist_next_, built_, cnt_, build_child_, blo_, bhi_, chunk_off_, gh_max_;
  at::Tensor scan_status_, scan_ticket_, scan_fault_, tile_cnt_, tile_off_, node_base_, node_r_;
  uint32_t scan_epoch_ = 0;
  // KDL_TUNE gbdt_route_scan (default 0): 1 = the fused route + look-back scan (one launch; measured
  // slower: 59.9 us per level against 23.0 + 14.6 for route_flags + the device scan, 941-952 vs
  // 1,053-1,064 boosting rounds/s at 2M x 28 -- the look-back's chain of cross-XCD atomic round trips
  // over 977 tiles; profiles/r06_gbdt_route_scan.txt); 0 = route_flags + a device scan
  // KDL_TUNE gbdt_route_plan (default 1): the three-launch level (route + counts, plan, partition)
  static bool route_plan_on() {
    if (g_route_plan < 0) g_route_plan = kdl::tune_int("gbdt_route_plan", 1);
    return g_route_plan != 0;
  }
  static bool route_scan_on() {
    if (g_route_scan < 0) g_route_scan = kdl::tune_int("gbdt_route_scan", 0);
    return g_route_scan != 0;
  }

 public:
  static int g_route_scan;
  static int g_route_plan;
};

int GbdtGrower::g_route_scan = -1;
int GbdtGrower::g_route_plan = -1;

// (flag, inclusive scan of flag) of one level's routing, by the fused route + look-back scan
// (``fused``) or by route_flags + a device scan: the test hook of route_scan_kernel.  ``calls``
// > 1 repeats the fused launch on one status array (epochs 1, 2, ...): the last result returned.
std::vector<at::Tensor> gbdt_route_scan_test(const at::Tensor& bins, const at::Tensor& rows,
                                             const at::Tensor& node_pos, const at::Tensor& split,
                                             const at::Tensor& t_feat, const at::Tensor& t_bin, int64_t h0,
                                             int64_t L, bool fused, int64_t calls, bool feature_major) {
  TORCH_CHECK(bins.is_cuda() && bins.scalar_type() == at::kByte && bins.dim() == 2 && bins.is_contiguous(),
              "gbdt_route_scan_test: uint8 bins [N, F]");
  for (const at::Tensor* t : {&rows, &node_pos, &split, &t_feat, &t_bin})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kInt && t->is_contiguous(), "gbdt_route_scan_test: int32");
  const int n = static_cast<int>(rows.numel()), F = static_cast<int>(bins.size(1));
  TORCH_CHECK(node_pos.numel() == n && split.numel() >= L && t_feat.numel() >= h0 + L && t_bin.numel() >= h0 + L,
              "gbdt_route_scan_test: sizes");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(bins.device());
  auto flag = at::empty({n}, rows.options()), sc = at::empty({n}, rows.options());
  if (!fused) {
    at::Tensor b = feature_major ? bins.t().contiguous() : bins;
    ck(kdl::gbdt_route_flags(b.data_ptr<uint8_t>(), ip(rows), ip(node_pos), ip(split), ip(t_feat), ip(t_bin), F,
                             n, static_cast<int>(h0), static_cast<int>(L), ip(flag), stream(), feature_major),
       "gbdt_route_flags");
    at::cumsum_out(sc, flag, 0, at::kInt);
    return {flag, sc};
  }
  auto status = at::zeros({std::max(1, kdl::gbdt_route_scan_tiles(n))}, rows.options().dtype(at::kLong));
  auto ticket = at::zeros({1}, rows.options()), fault = at::zeros({1}, rows.options());
  for (int64_t c = 1; c <= std::max<int64_t>(calls, 1); ++c)
    ck(kdl::gbdt_route_scan(bins.data_ptr<uint8_t>(), ip(rows), ip(node_pos), ip(split), ip(t_feat), ip(t_bin), F, n,
                            static_cast<int>(h0), static_cast<int>(L), ip(flag), ip(sc),
                            reinterpret_cast<unsigned long long*>(status.data_ptr<int64_t>()),
                            reinterpret_cast<unsigned*>(ip(ticket)), static_cast<uint32_t>(c), ip(fault), stream()),
       "gbdt_route_scan");
  TORCH_CHECK(fault.item<int>() == 0, "gbdt_route_scan_test: look-back timeouts");
  TORCH_CHECK(ticket.item<int>() == 0, "gbdt_route_scan_test: the tile ticket was not re-armed");
  return {flag, sc};
}

// One level's (rows_next, node_pos_next, lo_next, hi_next, child counts) by the three-launch path
// (``plan``) or by route_flags + scan + partition + children: the test hook of gbdt_route_partition.
std::vector<at::Tensor> gbdt_level_test(const at::Tensor& bins, const at::Tensor& rows, const at::Tensor& node_pos,
                                        const at::Tensor& split, const at::Tensor& t_feat, const at::Tensor& t_bin,
                                        const at::Tensor& lo, const at::Tensor& hi, int64_t h0, int64_t L, bool plan) {
  TORCH_CHECK(bins.is_cuda() && bins.scalar_type() == at::kByte && bins.dim() == 2 && bins.is_contiguous(),
              "gbdt_level_test: uint8 bins [N, F]");
  for (const at::Tensor* t : {&rows, &node_pos, &split, &t_feat, &t_bin, &lo, &hi})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kInt && t->is_contiguous(), "gbdt_level_test: int32");
  const int n = static_cast<int>(rows.numel()), F = static_cast<int>(bins.size(1));
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(bins.device());
  auto io = rows.options();
  auto rn = at::empty({n}, io), pn = at::empty({n}, io), flag = at::empty({n}, io);
  auto lon = at::zeros({2 * L}, io), hin = at::zeros({2 * L}, io), bc = at::zeros({L}, io);
  auto blo = at::zeros({L}, io), bhi = at::zeros({L}, io);
  auto cnt = at::zeros({2 * L}, io.dtype(at::kFloat));
  if (plan) {
    auto bt = bins.t().contiguous();
    const int nt = std::max(1, kdl::gbdt_level_tiles(n));
    auto tc = at::empty({nt}, io), to = at::empty({nt}, io), ti = at::empty({n}, io);
    auto nb = at::empty({L}, io), nrr = at::empty({L}, io);
    ck(kdl::gbdt_route_partition(bt.data_ptr<uint8_t>(), true, F, ip(rows), ip(node_pos), ip(split), ip(t_feat),
                                 ip(t_bin), ip(lo), ip(hi), n, static_cast<int>(h0), static_cast<int>(L), ip(flag),
                                 ip(ti), ip(tc), ip(to), ip(nb), ip(nrr), ip(rn), ip(pn), ip(lon), ip(hin), fp(cnt), 1,
                                 ip(bc), ip(blo), ip(bhi), stream()),
       "gbdt_route_partition");
  } else {
    auto sc = at::empty({n}, io);
    ck(kdl::gbdt_route_flags(bins.data_ptr<uint8_t>(), ip(rows), ip(node_pos), ip(split), ip(t_feat), ip(t_bin), F, n,
                             static_cast<int>(h0), static_cast<int>(L), ip(flag), stream()),
       "gbdt_route_flags");
    at::cumsum_out(sc, flag, 0, at::kInt);
    ck(kdl::gbdt_partition(ip(rows), ip(node_pos), ip(split), ip(lo), ip(hi), ip(flag), ip(sc), n,
                           static_cast<int>(h0), static_cast<int>(L), ip(rn), ip(pn), stream()),
       "gbdt_partition");
    ck(kdl::gbdt_children(ip(split), ip(lo), ip(hi), ip(sc), static_cast<int>(L), ip(lon), ip(hin), fp(cnt), 1,
                          ip(bc), ip(blo), ip(bhi), stream()),
       "gbdt_children");
  }
  return {rn, pn, lon, hin, cnt, bc, blo, bhi};
}

at::Tensor gbdt_quantise(const at::Tensor& X, const at::Tensor& cuts, int64_t num_bins) {
  TORCH_CHECK(X.is_cuda() && X.dim() == 2, "gbdt_quantise: X [N, F] on the GPU");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(X.device());
  auto x = X.to(at::kFloat).contiguous();
  // the cuts may come from a host fit (fit_cuts on a CPU X): the kernel reads them on X's device
  auto c = cuts.to(X.device(), at::kFloat).contiguous();
  TORCH_CHECK(c.dim() == 2 && c.size(0) == x.size(1), "gbdt_quantise: cuts [F, ncut]");
  TORCH_CHECK(num_bins >= 2 && num_bins <= 256, "gbdt_quantise: 2 <= num_bins <= 256");
  auto out = at::empty(x.sizes(), x.options().dtype(at::kByte));
  ck(kdl::gbdt_quantise(fp(x), fp(c), x.size(0), static_cast<int>(x.size(1)), static_cast<int>(c.size(1)),
                        static_cast<int>(num_bins - 1), out.data_ptr<uint8_t>(), stream()),
     "gbdt_quantise");
  return out;
}

}  // namespace

void register_gbdt(pybind11::module& m) {
  namespace py = pybind11;
  py::class_<GbdtGrower>(m, "GbdtGrower")
      .def(py::init<const at::Tensor&, const at::Tensor&, int64_t, int64_t, double, double, double, double>(),
           py::arg("bins"), py::arg("cuts"), py::arg("num_bins"), py::arg("max_depth"), py::arg("reg_lambda"),
           py::arg("gamma"), py::arg("learning_rate"), py::arg("min_child_weight"))
      .def("begin_tree", &GbdtGrower::begin_tree)
      .def("level_a", &GbdtGrower::level_a)
      .def("level_b", &GbdtGrower::level_b)
      .def("level_c", &GbdtGrower::level_c)
      .def("grow_local", &GbdtGrower::grow_local)
      .def("node_of_row", &GbdtGrower::node_of_row)
      .def("add_leaf", &GbdtGrower::add_leaf)
      .def("heap_packed", &GbdtGrower::heap_packed)
      .def("tree", &GbdtGrower::tree)
      .def("stats", &GbdtGrower::stats)
      .def("rows_per_chunk", &GbdtGrower::rows_per_chunk)
      .def("scan_faults", &GbdtGrower::scan_faults)
      .def_static("set_route_plan", [](int v) { GbdtGrower::g_route_plan = v; },
                  "1: the three-launch level (route + counts, plan, partition), 0: route / scan / partition / "
                  "children, -1: KDL_TUNE gbdt_route_plan")
      .def_static("set_route_scan", [](int v) { GbdtGrower::g_route_scan = v; },
                  "1: fused route + look-back scan, 0: route_flags + device scan, -1: KDL_TUNE gbdt_route_scan");
  m.def("gbdt_quantise", &gbdt_quantise, "GBDT feature quantisation (bins = #cuts < x, clamped)");
  m.def("gbdt_level_test", &gbdt_level_test, "one level's partition + child segments: three-launch plan or scan path");
  m.def("gbdt_route_scan_test", &gbdt_route_scan_test, "(flag, inclusive scan) of a level's routing: fused or two-pass",
        py::arg("bins"), py::arg("rows"), py::arg("node_pos"), py::arg("split"), py::arg("t_feat"), py::arg("t_bin"),
        py::arg("h0"), py::arg("L"), py::arg("fused"), py::arg("calls") = 1, py::arg("feature_major") = false);
}
