// Native A/B knobs, all in ONE environment variable:
//   KDL_TUNE="gemm_cfg=5,igemm_rounds=2,halo=0"
// tune_int(name, dflt) is the integer after "name=" in KDL_TUNE (dflt when the
// key is absent); tune_has(name) tells whether the key is present.  Keys
// (defaults are the measured winners, docs/perf_notes.md):
//   gemm_rounds, gemm_cfg, gemm_core (-1 by shape, 0 register-staged, 1 LDS-DMA),
//   igemm_rounds, igemm_cfg, igemm_price (timing only: 1 drops A's loads, 2 B's),
//   wgrad_big, wgrad_blocks, wgrad_red_blocks, price_wgrad_reduce (timing only: 0 skips),
//   halo, halo_pro, halo_wg_blocks, bn_min_rows, igemm_n256, gbdt_rpb, gbdt_unroll, gbdt_ftile,
//   gbdt_hist_rows, gbdt_route_scan, gbdt_route_plan, gbdt_pack64, gbdt_price_noflush (timing only), gram_blocks,
//   ctr_tile (CTR GEMM tile, -1 by shape), ctr_igemm, ctr_igemm_cfg, ctr_handoff, ctr_head_rpb (docs/startup_flags.md).
#pragma once

#include <cstdlib>
#include <cstring>

namespace kdl {

inline const char* tune_find(const char* name) {
  const char* spec = getenv("KDL_TUNE");
  if (!spec || !*spec) return nullptr;
  const size_t n = strlen(name);
  for (const char* p = spec; *p;) {
    while (*p == ',' || *p == ' ') ++p;
    if (strncmp(p, name, n) == 0 && p[n] == '=') return p + n + 1;
    while (*p && *p != ',') ++p;
  }
  return nullptr;
}

inline bool tune_has(const char* name) { return tune_find(name) != nullptr; }

inline int tune_int(const char* name, int dflt) {
  const char* v = tune_find(name);
  return v ? atoi(v) : dflt;
}

}  // namespace kdl
