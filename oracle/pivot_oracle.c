/*
 * pivot_oracle.c — CPU restatement of the reference placement policies. TEST INFRASTRUCTURE.
 *
 * This file is the parity checker, not the product. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it. The product path (pivot_place) never links or calls
 * it and fails loudly when its HIP library is missing.
 *
 * It restates, loop for loop, the schedule() bodies of the reference (Python) policies on the
 * SoA round layout of include/pivot_place.h, with all pointers in HOST memory:
 *
 *   cost_aware  scheduler/cost_aware.py:28-43 (group loop), :60-61 (_sort_tasks),
 *               :63-97 (_best_fit), :99-127 (_first_fit)
 *   opportunistic  scheduler/opportunistic.py:11-20
 *   vbp         scheduler/vbp.py:13-29 (first-fit), :39-50 (best-fit)
 *
 * Grouping and anchor choice (cost_aware.py:45-58 and the randomizer.choice at :38-39) stay in
 * the Python caller, as they do for the GPU path; groups arrive as task_group/group_anchor.
 *
 * Arithmetic (pinned against the golden fixtures, tests/golden/):
 *   - ||x||2 = sqrt(s), s = fma(x3,x3, fma(x2,x2, fma(x1,x1, fma(x0,x0, 0)))): numpy
 *     la.norm(x, 2) is sqrt(x.dot(x)) and OpenBLAS ddot runs that FMA chain for n = 4.
 *   - fit tests compare elementwise, as np.all(resc >= d) / np.all(r > d) do.
 *   - commits are resc[h] -= d, elementwise fp64.
 *   - RandomState.choice(n) == randint(0, n): no draw when n == 1, else 32-bit MT19937
 *     outputs masked to the next power of two minus one and rejected while > n - 1.
 * Compile with -ffp-contract=off and without -ffast-math.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "pivot_place.h"

/* ---------------------------------------------------------------- arithmetic helpers */
double oracle_norm4(const double x[4]) {
  double s = fma(x[0], x[0], 0.0);
  s = fma(x[1], x[1], s);
  s = fma(x[2], x[2], s);
  s = fma(x[3], x[3], s);
  return sqrt(s);
}

static inline void host_vec(const double* avail, int H, int h, double a[4]) {
  a[0] = avail[h]; a[1] = avail[H + h]; a[2] = avail[2 * H + h]; a[3] = avail[3 * H + h];
}
static inline void task_vec(const double* dem, int T, int t, double d[4]) {
  d[0] = dem[t]; d[1] = dem[T + t]; d[2] = dem[2 * T + t]; d[3] = dem[3 * T + t];
}
static inline int fits_ge(const double a[4], const double d[4]) {
  return a[0] >= d[0] && a[1] >= d[1] && a[2] >= d[2] && a[3] >= d[3];
}
static inline int fits_gt(const double a[4], const double d[4]) {
  return a[0] > d[0] && a[1] > d[1] && a[2] > d[2] && a[3] > d[3];
}
static inline void commit(double* avail, int H, int h, const double d[4]) {
  avail[h] -= d[0]; avail[H + h] -= d[1]; avail[2 * H + h] -= d[2]; avail[3 * H + h] -= d[3];
}

/* ---------------------------------------------------------------- MT19937 (numpy legacy) */
#define MT_N 624
#define MT_M 397
static void mt_twist(uint32_t* key) {
  for (int i = 0; i < MT_N; i++) {
    uint32_t y = (key[i] & 0x80000000u) | (key[(i + 1) % MT_N] & 0x7fffffffu);
    uint32_t v = key[(i + MT_M) % MT_N] ^ (y >> 1);
    if (y & 1u) v ^= 0x9908b0dfu;
    key[i] = v;
  }
}
static uint32_t mt_next(uint32_t* st) {
  uint32_t* key = st;
  if (st[MT_N] >= MT_N) { mt_twist(key); st[MT_N] = 0; }
  uint32_t y = key[st[MT_N]++];
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}
/* RandomState.randint(0, n) for 1 <= n <= 2^32 (numpy legacy masked rejection). */
uint32_t oracle_randint(uint32_t* st, uint64_t n) {
  uint64_t rng = n - 1;
  if (rng == 0) return 0;
  if (rng == 0xffffffffu) return mt_next(st);
  uint32_t mask = (uint32_t)rng;
  mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
  uint32_t v;
  while ((v = (mt_next(st) & mask)) > (uint32_t)rng) {}
  return v;
}

/* ---------------------------------------------------------------- stable orderings */
typedef struct { double k; int32_t i; } keyed;
static int cmp_keyed(const void* a, const void* b) {   /* (k asc, i asc): a stable sort */
  const keyed* x = (const keyed*)a; const keyed* y = (const keyed*)b;
  if (x->k < y->k) return -1;
  if (x->k > y->k) return 1;
  return (x->i > y->i) - (x->i < y->i);
}

/* Tasks of group g (caller order), then stably sorted by -||d||2 (cost_aware.py:60-61,
 * vbp.py:28-29,42). Writes into out, returns count. */
static int group_tasks(const pvt_round* r, int g, int sort, keyed* scratch, int32_t* out) {
  int T = r->n_tasks, n = 0;
  for (int t = 0; t < T; t++)
    if (!r->task_group || r->task_group[t] == g) {
      double d[4]; task_vec(r->dem, T, t, d);
      scratch[n].k = -oracle_norm4(d);
      scratch[n].i = t;
      n++;
    }
  if (sort) qsort(scratch, (size_t)n, sizeof(keyed), cmp_keyed);
  for (int j = 0; j < n; j++) out[j] = scratch[j].i;
  return n;
}

/* The bandwidth of cost_aware's host_score_func (cost_aware.py:73-79, :106-112): the static
 * in_route.bw + out_route.bw = bw[a][z] + bw[z][a], or with realtime_bw the caller's
 * in_route.realtime_bw + out_route.realtime_bw of group g and host h. */
static inline double ca_bw(const pvt_round* r, int g, int anchor, int h) {
  const int Z = r->n_zones, z = r->zone[h];
  if (r->rt_bw) return r->rt_bw[(size_t)g * r->n_hosts + h];
  return r->bw[anchor * Z + z] + r->bw[z * Z + anchor];
}

/* ---------------------------------------------------------------- policies */
/* cost_aware _first_fit (cost_aware.py:99-127). */
static void ca_first_fit(const pvt_round* r, const int32_t* tasks, int n, int g, int anchor,
                         keyed* hs) {
  int H = r->n_hosts, T = r->n_tasks, Z = r->n_zones;
  for (int h = 0; h < H; h++) { hs[h].i = h; hs[h].k = 0.0; }
  if (r->sort_hosts) {
    /* host_score_func (:104-116): c * df / (r * bw), keys frozen for the group (:118-119). */
    for (int h = 0; h < H; h++) {
      double a[4]; host_vec(r->avail, H, h, a);
      double rn = oracle_norm4(a);
      int z = r->zone[h];
      double bw = ca_bw(r, g, anchor, h);
      double c = r->cost[anchor * Z + z] + r->cost[z * Z + anchor];
      double df = r->decay ? (double)r->decay[h] : 1.0;
      hs[h].k = c * df / (rn * bw);
    }
    qsort(hs, (size_t)H, sizeof(keyed), cmp_keyed);
  }
  for (int j = 0; j < n; j++) {
    int t = tasks[j];
    double d[4]; task_vec(r->dem, T, t, d);
    for (int q = 0; q < H; q++) {
      int h = hs[q].i;
      double a[4]; host_vec(r->avail, H, h, a);
      if (fits_gt(a, d)) {                       /* np.all(r > t_demand) (:124) */
        r->placement[t] = h;
        commit(r->avail, H, h, d);
        break;
      }
    }
  }
}

/* cost_aware _best_fit (cost_aware.py:63-97); host_decay is rejected by the caller. */
static void ca_best_fit(const pvt_round* r, const int32_t* tasks, int n, int g, int anchor) {
  int H = r->n_hosts, T = r->n_tasks, Z = r->n_zones;
  for (int j = 0; j < n; j++) {
    int t = tasks[j];
    double d[4]; task_vec(r->dem, T, t, d);
    int best = -1; double bs = 0.0;
    for (int h = 0; h < H; h++) {
      double a[4]; host_vec(r->avail, H, h, a);
      if (!fits_ge(a, d)) continue;              /* np.all(resc >= t_demand) (:87) */
      double x[4] = {a[0] - d[0], a[1] - d[1], a[2] - d[2], a[3] - d[3]};
      double rn = oracle_norm4(x);
      int z = r->zone[h];
      double bw = ca_bw(r, g, anchor, h);
      double c = r->cost[anchor * Z + z] + r->cost[z * Z + anchor];
      double s = c * rn * 1.0 / bw;              /* t * r * decay / bw (:83), decay == 1 */
      if (best < 0 || s < bs) { best = h; bs = s; }   /* min(): first minimum (:92) */
    }
    if (best >= 0) { r->placement[t] = best; commit(r->avail, H, best, d); }
  }
}

/* opportunistic (opportunistic.py:11-20). */
static void opportunistic(const pvt_round* r, int32_t* order) {
  int H = r->n_hosts, T = r->n_tasks;
  for (int t = 0; t < T; t++) {
    order[t] = t;
    double d[4]; task_vec(r->dem, T, t, d);
    int64_t nq = 0;
    for (int h = 0; h < H; h++) { double a[4]; host_vec(r->avail, H, h, a); nq += fits_ge(a, d); }
    if (nq == 0) continue;
    uint32_t k = oracle_randint(r->mt_state, (uint64_t)nq);
    for (int h = 0; h < H; h++) {
      double a[4]; host_vec(r->avail, H, h, a);
      if (fits_ge(a, d)) {
        if (k == 0) { r->placement[t] = h; commit(r->avail, H, h, d); break; }
        k--;
      }
    }
  }
}

/* vbp first-fit (vbp.py:13-26). */
static void vbp_first_fit(const pvt_round* r, const int32_t* tasks, int n) {
  int H = r->n_hosts, T = r->n_tasks;
  for (int j = 0; j < n; j++) {
    int t = tasks[j];
    double d[4]; task_vec(r->dem, T, t, d);
    for (int h = 0; h < H; h++) {
      double a[4]; host_vec(r->avail, H, h, a);
      if (fits_ge(a, d)) { r->placement[t] = h; commit(r->avail, H, h, d); break; }
    }
  }
}

/* vbp best-fit (vbp.py:39-50): min of (||r - d||, host_id) over r > d. */
static void vbp_best_fit(const pvt_round* r, const int32_t* tasks, int n) {
  int H = r->n_hosts, T = r->n_tasks;
  for (int j = 0; j < n; j++) {
    int t = tasks[j];
    double d[4]; task_vec(r->dem, T, t, d);
    int best = -1; double bs = 0.0; uint32_t bt = 0;
    for (int h = 0; h < H; h++) {
      double a[4]; host_vec(r->avail, H, h, a);
      if (!fits_gt(a, d)) continue;
      double x[4] = {a[0] - d[0], a[1] - d[1], a[2] - d[2], a[3] - d[3]};
      double s = oracle_norm4(x);
      uint32_t tb = r->tiebreak[h];
      if (best < 0 || s < bs || (s == bs && tb < bt)) { best = h; bs = s; bt = tb; }
    }
    if (best >= 0) { r->placement[t] = best; commit(r->avail, H, best, d); }
  }
}

/* Same contract as pvt_place, host pointers. */
int oracle_place(const pvt_round* r) {
  if (!r || r->n_hosts < 1 || r->n_tasks < 0 || r->n_zones < 1) return PVT_EINVAL;
  if (r->n_tasks == 0) return PVT_OK;
  if (!r->avail || !r->zone || !r->dem || !r->placement || !r->order) return PVT_EINVAL;
  int H = r->n_hosts, T = r->n_tasks;
  for (int t = 0; t < T; t++) r->placement[t] = -1;
  keyed* ks = (keyed*)malloc(sizeof(keyed) * (size_t)(H > T ? H : T));
  if (!ks) return PVT_ENOMEM;
  int rc = PVT_OK;
  switch (r->mode) {
    case PVT_CA_FF:
    case PVT_CA_BF: {
      if (!r->cost || !r->bw) { rc = PVT_EINVAL; break; }
      int G = r->task_group ? r->n_groups : 1, off = 0;
      if (r->task_group && !r->group_anchor) { rc = PVT_EINVAL; break; }
      for (int g = 0; g < G; g++) {
        int anchor = r->group_anchor ? r->group_anchor[g] : 0;
        int n = group_tasks(r, g, r->sort_tasks, ks, r->order + off);
        keyed* hs = (keyed*)malloc(sizeof(keyed) * (size_t)H);
        if (!hs) { rc = PVT_ENOMEM; break; }
        if (r->mode == PVT_CA_FF) ca_first_fit(r, r->order + off, n, g, anchor, hs);
        else ca_best_fit(r, r->order + off, n, g, anchor);
        free(hs);
        off += n;
      }
      break;
    }
    case PVT_OPP:
      if (!r->mt_state) { rc = PVT_EINVAL; break; }
      opportunistic(r, r->order);
      break;
    case PVT_VBP_FF:
    case PVT_VBP_BF: {
      int n = group_tasks(r, 0, r->sort_tasks, ks, r->order);
      if (r->mode == PVT_VBP_FF) vbp_first_fit(r, r->order, n);
      else if (!r->tiebreak) rc = PVT_EINVAL;
      else vbp_best_fit(r, r->order, n);
      break;
    }
    default:
      rc = PVT_EINVAL;
  }
  free(ks);
  return rc;
}

/* ---------------------------------------------------------------- multi-threaded baseline */
/*
 * oracle_place_mt: the same restatement with every per-task host scan split over `threads`
 * OpenMP threads (static contiguous chunks), each chunk reduced to its first best host and the
 * chunks combined in host order, then the commit applied serially -- so results are identical
 * to oracle_place's (tests/test_oracle_golden.py checks it). bench.py times it as the all-cores
 * CPU baseline; it is not a parity checker.
 */
#include <omp.h>

/* Scans of fewer hosts stay on one thread: a parallel region per task costs more than the
 * scan (and stalls under CPU contention), so the all-cores baseline of small rounds is the
 * 1-thread one. */
#define MT_MIN_HOSTS 4096

typedef struct { double s; uint32_t tb; int32_t h; } cand;
static inline int cand_less(cand a, cand b) {   /* (s, tb, h) lexicographic; h < 0 = none */
  if (a.h < 0) return 0;
  if (b.h < 0) return 1;
  if (a.s != b.s) return a.s < b.s;
  if (a.tb != b.tb) return a.tb < b.tb;
  return a.h < b.h;
}

/* Best host of one task: mode CA_BF (>=, egress score), VBP_BF (>, norm, tiebreak), first-fit
 * by index (strict or not), or first-fit over hosts in `hs` key order (CA_FF sort_hosts). */
static int32_t mt_pick(const pvt_round* r, int mode, const double d[4], int g, int anchor,
                       const keyed* hs, int threads) {
  const int H = r->n_hosts, Z = r->n_zones;
  cand best = {0.0, 0u, -1};
#pragma omp parallel num_threads(threads) if (H >= MT_MIN_HOSTS)
  {
    cand mine = {0.0, 0u, -1};
#pragma omp for schedule(static) nowait
    for (int q = 0; q < H; q++) {
      const int h = hs ? hs[q].i : q;
      double a[4]; host_vec(r->avail, H, h, a);
      if (mode == PVT_CA_BF) {
        if (!fits_ge(a, d)) continue;
        double x[4] = {a[0] - d[0], a[1] - d[1], a[2] - d[2], a[3] - d[3]};
        int z = r->zone[h];
        double bw = ca_bw(r, g, anchor, h);
        double c = r->cost[anchor * Z + z] + r->cost[z * Z + anchor];
        cand k = {c * oracle_norm4(x) * 1.0 / bw, 0u, h};
        if (cand_less(k, mine)) mine = k;
      } else if (mode == PVT_VBP_BF) {
        if (!fits_gt(a, d)) continue;
        double x[4] = {a[0] - d[0], a[1] - d[1], a[2] - d[2], a[3] - d[3]};
        cand k = {oracle_norm4(x), r->tiebreak[h], h};
        if (cand_less(k, mine)) mine = k;
      } else {   /* first fit: the first position q in scan order */
        const int strict = (mode == PVT_CA_FF);
        if (mine.h >= 0) continue;
        if (strict ? fits_gt(a, d) : fits_ge(a, d)) { mine.s = (double)q; mine.h = h; }
      }
    }
#pragma omp critical
    if (cand_less(mine, best)) best = mine;
  }
  return best.h;
}

int oracle_place_mt(const pvt_round* r, int threads) {
  if (!r || r->n_hosts < 1 || r->n_tasks < 0 || r->n_zones < 1) return PVT_EINVAL;
  if (threads < 1) threads = 1;
  if (r->n_tasks == 0) return PVT_OK;
  if (!r->avail || !r->zone || !r->dem || !r->placement || !r->order) return PVT_EINVAL;
  const int H = r->n_hosts, T = r->n_tasks, Z = r->n_zones;
  if (r->mode == PVT_OPP) {
    if (!r->mt_state) return PVT_EINVAL;
    for (int t = 0; t < T; t++) {
      r->order[t] = t;
      r->placement[t] = -1;
      double d[4]; task_vec(r->dem, T, t, d);
      int64_t nq = 0;
#pragma omp parallel for num_threads(threads) reduction(+ : nq) schedule(static) if (H >= MT_MIN_HOSTS)
      for (int h = 0; h < H; h++) { double a[4]; host_vec(r->avail, H, h, a); nq += fits_ge(a, d); }
      if (nq == 0) continue;
      uint32_t k = oracle_randint(r->mt_state, (uint64_t)nq);
      for (int h = 0; h < H; h++) {
        double a[4]; host_vec(r->avail, H, h, a);
        if (fits_ge(a, d)) {
          if (k == 0) { r->placement[t] = h; commit(r->avail, H, h, d); break; }
          k--;
        }
      }
    }
    return PVT_OK;
  }
  for (int t = 0; t < T; t++) r->placement[t] = -1;
  keyed* ks = (keyed*)malloc(sizeof(keyed) * (size_t)(H > T ? H : T));
  keyed* hs = (keyed*)malloc(sizeof(keyed) * (size_t)H);
  if (!ks || !hs) { free(ks); free(hs); return PVT_ENOMEM; }
  const int ca = r->mode == PVT_CA_FF || r->mode == PVT_CA_BF;
  if (ca && (!r->cost || !r->bw || (r->task_group && !r->group_anchor))) { free(ks); free(hs); return PVT_EINVAL; }
  if (r->mode == PVT_VBP_BF && !r->tiebreak) { free(ks); free(hs); return PVT_EINVAL; }
  const int G = (ca && r->task_group) ? r->n_groups : 1;
  int off = 0;
  for (int g = 0; g < G; g++) {
    const int anchor = (ca && r->group_anchor) ? r->group_anchor[g] : 0;
    const int n = group_tasks(r, ca ? g : 0, r->sort_tasks, ks, r->order + off);
    const keyed* order = NULL;
    if (r->mode == PVT_CA_FF && r->sort_hosts) {   /* frozen keys of the group (:104-119) */
#pragma omp parallel for num_threads(threads) schedule(static) if (H >= MT_MIN_HOSTS)
      for (int h = 0; h < H; h++) {
        double a[4]; host_vec(r->avail, H, h, a);
        int z = r->zone[h];
        double bw = ca_bw(r, g, anchor, h);
        double c = r->cost[anchor * Z + z] + r->cost[z * Z + anchor];
        double df = r->decay ? (double)r->decay[h] : 1.0;
        hs[h].i = h;
        hs[h].k = c * df / (oracle_norm4(a) * bw);
      }
      qsort(hs, (size_t)H, sizeof(keyed), cmp_keyed);
      order = hs;
    }
    for (int j = 0; j < n; j++) {
      const int t = r->order[off + j];
      double d[4]; task_vec(r->dem, T, t, d);
      const int32_t h = mt_pick(r, r->mode, d, g, anchor, order, threads);
      if (h >= 0) { r->placement[t] = h; commit(r->avail, H, h, d); }
    }
    off += n;
  }
  free(ks);
  free(hs);
  return PVT_OK;
}

/* ---------------------------------------------------------------- anchor resolution (a3)
 * CostAwareGlobalScheduler._group_tasks (scheduler/cost_aware.py:45-58), per item:
 *   placement, _ = max(Counter(list).items(), key=lambda x: x[1])
 * Counter's items() follow first insertion and max() keeps the first maximum. Entries are host
 * indices (-1 = no placement) or, with inst_host, indices into it. Outputs as pvt_anchor():
 * anchor_zone -1 empty list, -2 mode entry -1, -3 invalid item (returns PVT_EINVAL). */
int oracle_anchor(int32_t C, int32_t H, const int64_t* off, const int32_t* list,
                  const int32_t* inst_host, int64_t n_inst, const int32_t* zone,
                  int32_t* mode_host, int32_t* anchor_zone) {
  int64_t* count = (int64_t*)calloc((size_t)H + 1, sizeof(int64_t));
  int bad = 0;
  if (!count) return PVT_ENOMEM;
  for (int32_t c = 0; c < C; ++c) {
    const int64_t lo = off[c], hi = off[c + 1];
    int ok = lo >= 0 && hi >= lo;
    for (int64_t j = lo; ok && j < hi; ++j) {
      int32_t h = list[j];
      if (inst_host) { if (h < 0 || h >= n_inst) { ok = 0; break; } h = inst_host[h]; }
      if (h < -1 || h >= H) ok = 0;
    }
    if (!ok) { mode_host[c] = -1; anchor_zone[c] = -3; ++bad; continue; }
    if (hi == lo) { mode_host[c] = -1; anchor_zone[c] = -1; continue; }
    int32_t best = 0; int64_t best_n = -1;
    for (int64_t j = lo; j < hi; ++j) {                 /* Counter(list) */
      int32_t h = inst_host ? inst_host[list[j]] : list[j];
      count[h + 1] += 1;
    }
    for (int64_t j = lo; j < hi; ++j) {                 /* max over items() in insertion order */
      int32_t h = inst_host ? inst_host[list[j]] : list[j];
      if (count[h + 1] > best_n) { best_n = count[h + 1]; best = h; }
      if (count[h + 1] > 0) count[h + 1] = -count[h + 1];   /* visit each key once */
    }
    for (int64_t j = lo; j < hi; ++j) {
      int32_t h = inst_host ? inst_host[list[j]] : list[j];
      count[h + 1] = 0;
    }
    mode_host[c] = best;
    anchor_zone[c] = best >= 0 ? zone[best] : -2;
  }
  free(count);
  return bad ? PVT_EINVAL : PVT_OK;
}

/* ---------------------------------------------------------------- meter aggregates (f4)
 * resources/meter.py:31-53, left to right exactly as the reference's Python sums run:
 *   cumulative_instance_hours = sum([sum([v[1]-v[0] for v in vals]) for h, vals in hosts])/3600
 *   total_network_traffic_cost: cost += meta.cost[src, dst] * data_size / 8000 per route, with
 *     data_size = sum([sum(size for transfers) for packets])
 *   average_congestion_delay: delay += start_i - end_{i-1} over every packet's transfers,
 *     n_pkts and delay / n_pkts
 * Host pointers, layout of pvt_meter_log. Returns PVT_EINVAL on an out-of-range offset. */
int oracle_meter(const pvt_meter_log* m) {
  for (int32_t s = 0; s < m->n_scen; ++s) {
    const int64_t h0 = m->host_off[s], h1 = m->host_off[s + 1];
    const int64_t r0 = m->route_off[s], r1 = m->route_off[s + 1];
    if (h0 < 0 || h1 < h0 || h1 > m->n_host_rows || r0 < 0 || r1 < r0 || r1 > m->n_routes)
      return PVT_EINVAL;
    double hours = 0.0;
    for (int64_t h = h0; h < h1; ++h) {
      const int64_t v0 = m->iv_off[h], v1 = m->iv_off[h + 1];
      if (v0 < 0 || v1 < v0 || v1 > m->n_iv) return PVT_EINVAL;
      double acc = 0.0;
      for (int64_t v = v0; v < v1; ++v) acc += m->iv_end[v] - m->iv_start[v];
      hours += acc;
    }
    double cost = 0.0, delay = 0.0;
    int64_t npk = 0;
    for (int64_t r = r0; r < r1; ++r) {
      const int64_t p0 = m->pkt_off[r], p1 = m->pkt_off[r + 1];
      if (p0 < 0 || p1 < p0 || p1 > m->n_pkts) return PVT_EINVAL;
      double size = 0.0;
      for (int64_t p = p0; p < p1; ++p) {
        const int64_t t0 = m->tr_off[p], t1 = m->tr_off[p + 1];
        if (t0 < 0 || t1 < t0 || t1 > m->n_tr) return PVT_EINVAL;
        double ps = 0.0;
        for (int64_t t = t0; t < t1; ++t) ps += m->tr_size[t];
        size += ps;
      }
      cost += m->route_cost[r] * size / 8000.0;
    }
    for (int64_t r = r0; r < r1; ++r) {           /* average_congestion_delay's own loop */
      const int64_t p0 = m->pkt_off[r], p1 = m->pkt_off[r + 1];
      npk += p1 - p0;
      for (int64_t p = p0; p < p1; ++p)
        for (int64_t t = m->tr_off[p] + 1; t < m->tr_off[p + 1]; ++t)
          delay += m->tr_start[t] - m->tr_end[t - 1];
    }
    m->instance_hours[s] = hours / 3600.0;
    m->egress_cost[s] = cost;
    m->congestion_delay[s] = npk ? delay / (double)npk : 0.0;
  }
  return PVT_OK;
}
