/*
 * pivot_place.h — C ABI of the MI355X placement engine for the PIVOT simulator.
 *
 * One call, pvt_place(), runs one scheduling round of one policy: every ready task x host
 * candidate is scored on the GPU and a host is picked per task, with capacity commits applied
 * in the reference's sequential order. It replaces the body of the reference policies'
 * schedule() hook:
 *
 *   - scheduler/__init__.py:79-80   GlobalSchedulerBase.schedule(self, tasks)   (plugin hook)
 *   - scheduler/__init__.py:103     the per-round call site in _dispatch
 *   - scheduler/cost_aware.py:28-43, 60-127   PVT_CA_FF / PVT_CA_BF
 *   - scheduler/opportunistic.py:11-20        PVT_OPP
 *   - scheduler/vbp.py:13-29                  PVT_VBP_FF
 *   - scheduler/vbp.py:39-50                  PVT_VBP_BF
 *
 * The reference binds nothing natively (it is pure Python); the binding a maintainer adds is
 * a ctypes stub, shown in INTEGRATION.md and implemented in pivot_place/engine.py + _abi.py.
 *
 * Conventions
 *   - Plain C types only. Returns PVT_OK (0) or a negative PVT_E* code; never throws.
 *   - Array pointers in pvt_round are DEVICE pointers (HBM, e.g. from torch-ROCm tensors),
 *     except mt_state, which is host memory. The library never frees caller memory; scratch
 *     lives in the context and grows on demand.
 *   - Work is ordered on the context's stream; pvt_place() synchronises before it returns.
 *   - A context is not thread-safe. Use one per thread and per GPU.
 *   - Arithmetic is IEEE fp64 with no contraction, so results are bit-exact against the
 *     reference (squared norms are the sequential FMA chain numpy/OpenBLAS ddot performs).
 */
#ifndef PIVOT_PLACE_H
#define PIVOT_PLACE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PVT_ABI_VERSION 3

/* Return codes. */
#define PVT_OK            0
#define PVT_EINVAL       -1   /* bad argument (null pointer, size, mode)          */
#define PVT_ENODEV       -2   /* no usable gfx950 device                          */
#define PVT_EHIP         -3   /* a HIP runtime call failed (see pvt_last_error)   */
#define PVT_ENOMEM       -4   /* scratch allocation failed                        */
#define PVT_EUNSUPPORTED -5   /* configuration the engine does not implement      */
#define PVT_ESTALE       -6   /* pvt_shard_commit: the exchanged window was scored while the
                                 previous walk ran, and that walk stopped early -- call
                                 pvt_shard_score again (every rank gets it together)     */

/* Policies (kernel modes). */
enum pvt_mode {
  PVT_CA_FF  = 0, /* cost_aware first-fit: strict fit, hosts ordered by frozen per-group key
                     (sort_hosts) or by index; scheduler/cost_aware.py:99-127              */
  PVT_CA_BF  = 1, /* cost_aware best-fit: fit >=, min egress-cost x residual / bw;
                     scheduler/cost_aware.py:63-97                                         */
  PVT_OPP    = 2, /* opportunistic: fit >=, uniform pick by MT19937 randint;
                     scheduler/opportunistic.py:11-20                                      */
  PVT_VBP_FF = 3, /* vbp first-fit: fit >=, lowest index; scheduler/vbp.py:13-29          */
  PVT_VBP_BF = 4  /* vbp best-fit: strict fit, min residual norm, tie by host-id string;
                     scheduler/vbp.py:39-50                                                */
};

/*
 * One scheduling round. Sizes: H hosts, T ready tasks, Z zones, G groups.
 *
 * Host state is SoA: avail[r*H + h] for resource r in {0 cpus, 1 mem, 2 disk, 3 gpus}
 * (the snapshot of scheduler/__init__.py:82-85, in cluster.hosts order). Task demands are
 * SoA too: dem[r*T + t], in the order of the `tasks` list passed to schedule().
 *
 * Groups (cost_aware only, scheduler/cost_aware.py:45-58): task_group[t] in [0, G) and
 * group_anchor[g] is the anchor storage zone. Groups run in id order; tasks of a group in
 * caller order, stably sorted by descending ||d||2 when sort_tasks is set. For the other
 * policies pass task_group = NULL (one group holding every task).
 *
 * realtime_bw (cost_aware, scheduler/cost_aware.py:17,79,112): rt_bw[g*H + h] is the bandwidth
 * the reference uses instead of the static one for group g (0 without task_group) and host h,
 * in_route.realtime_bw + out_route.realtime_bw of the routes between g's anchor storage and h
 * (resources/network.py:70-73: 1 / ((queued MB + 1) / bw) per route, summed in that order). NULL:
 * the static bw[a][z] + bw[z][a].
 */
typedef struct pvt_round {
  int32_t mode;          /* enum pvt_mode                                                 */
  int32_t n_hosts;       /* H >= 1                                                        */
  int32_t n_tasks;       /* T >= 0                                                        */
  int32_t n_zones;       /* Z >= 1 (cost/bw are Z x Z)                                    */
  int32_t n_groups;      /* G (cost_aware); ignored when task_group is NULL               */
  int32_t sort_tasks;    /* stable sort by descending ||d||2 within each group            */
  int32_t sort_hosts;    /* PVT_CA_FF: order hosts by the frozen key (cost_aware.py:118)  */
  int32_t reserved;      /* must be 0                                                     */
  double* avail;         /* [4*H] in/out: commits are applied                             */
  const int32_t* zone;   /* [H] zone index of each host (Host.locality)                   */
  const uint32_t* tiebreak; /* [H] rank of the host-id string (PVT_VBP_BF), else NULL     */
  const int32_t* decay;  /* [H] max(len(h.tasks),1) (PVT_CA_FF host_decay), else NULL     */
  const double* cost;    /* [Z*Z] egress cost, cost[src*Z + dst] (ResourceMetadata.cost);
                            every cost[a][z] + cost[z][a] >= +0 (egress prices: a score
                            c*r/bw then never grows as a residual r shrinks, and 0 is the
                            least score). Host-array calls (pvt_place_host*) check both
                            contracts (PVT_EINVAL), device rounds must meet them          */
  const double* bw;      /* [Z*Z] jittered bandwidth, bw[src*Z + dst]; every bw[a][z] +
                            bw[z][a] > 0 (resources/network.py bandwidths are positive: the
                            engine orders cost_aware scores >= +0 by their bits)           */
  const double* dem;     /* [4*T] task demand (cpus, mem, disk, gpus)                     */
  const int32_t* task_group;   /* [T] or NULL                                             */
  const int32_t* group_anchor; /* [G] anchor zone per group, or NULL                      */
  int32_t* order;        /* [T] out: processing order (task indices)                      */
  int32_t* placement;    /* [T] out: host index, -1 = not placed (task stays waiting)     */
  uint32_t* mt_state;    /* HOST [625] in/out: MT19937 key[624] then pos (PVT_OPP)        */
  const double* rt_bw;   /* [G*H] realtime bandwidth per (group, host), or NULL (cost_aware) */
} pvt_round;

typedef struct pvt_ctx pvt_ctx;

/* Per-kernel-class timing gathered while profiling is on (HIP events on the ctx stream). */
typedef struct pvt_kstats {
  int64_t launches;      /* kernel launches timed                                         */
  double  ms;            /* summed device time, milliseconds                              */
  double  candidates;    /* task x host candidates those launches evaluated               */
  double  bytes;         /* algorithmic bytes: candidates x bytes/candidate (§8(d))       */
} pvt_kstats;

/* Kernel classes reported by pvt_get_kstats. */
enum pvt_kclass {
  PVT_K_SCORE = 0,   /* fused fit-mask + score + per-task top-K (the hot kernel)          */
  PVT_K_MERGE = 1,   /* per-task merge of segment top-K lists                              */
  PVT_K_COMMIT = 2,  /* sequential in-order commit walk                                    */
  PVT_K_OTHER = 3,   /* keys, norms, sorts, counts                                         */
  PVT_K_COUNT = 4
};

int  pvt_abi_version(void);
int  pvt_ctx_create(int device, pvt_ctx** out);
int  pvt_ctx_destroy(pvt_ctx* ctx);
/* Order the context's work on a caller stream (hipStream_t as void*), e.g.
 * torch.cuda.current_stream().cuda_stream. NULL is the device's default (null) stream, which is
 * what torch's default stream is. Until the first call the context uses a stream of its own. */
int  pvt_ctx_set_stream(pvt_ctx* ctx, void* stream);
int  pvt_place(pvt_ctx* ctx, const pvt_round* r);
/* Profiling: on = 1 records HIP events around every kernel launch (adds a little host overhead:
 * ~30 us per config-5 round of ~15 launches); on = 2 only around the named kernels of
 * pvt_get_kernel_kstats (the kernel-class times of the other launches stay zero). The events are
 * timing-only (hipEventDisableSystemFence) and come from a pool this call fills and records once
 * (synchronising the context's stream), so a timed round creates none. */
int  pvt_set_profiling(pvt_ctx* ctx, int on);
int  pvt_reset_kstats(pvt_ctx* ctx);
int  pvt_get_kstats(pvt_ctx* ctx, int kclass, pvt_kstats* out);
/* Per-kernel timing while profiling is on: the launches of the named __global__ kernel of the
 * placement path ("zwalk_kernel", "commit_kernel", "lwalk_kernel", "opp_commit_kernel",
 * "opp_count_kernel", "score_kernel", "band_score_kernel", "perm_scan_kernel", "ordered_kernel",
 * "resident_kernel", "merge_kernel", "merge_small_kernel", "merge_pkg_kernel",
 * "merge_path_kernel"), each bracketed
 * by its own HIP events on the stream it runs on. An unknown or unlaunched name gives zeros. */
int  pvt_get_kernel_kstats(pvt_ctx* ctx, const char* kernel, pvt_kstats* out);
/* With profiling on = 2, record events around the launches of this one named kernel only
 * (NULL or "": every named kernel). Each event pair costs the stream a few microseconds of idle
 * GPU (config 5: 0.33 ms of a 2.74 ms vbp best-fit round with every named kernel timed), so a
 * benchmark times only the kernel its roofline is about. */
int  pvt_set_profiling_kernel(pvt_ctx* ctx, const char* kernel);
/* Tuning knob: tasks per window (0 = the policy's default; capped at 1024). */
int  pvt_set_window(pvt_ctx* ctx, int tasks);
/* Tuning knob: tasks per wave of the best-fit score kernel, 0 (the policy's default: 2 for vbp
 * best-fit and for cost_aware below 262144 hosts, else 4), 2 or 4. Results are identical. */
int  pvt_set_score_tw(pvt_ctx* ctx, int tw);
/* Tuning knob: vbp best-fit rounds of at least min_hosts hosts (per shard) build their candidate
 * lists from a memory band over the hosts sorted once per round by snapshot memory (hosts
 * committed to since the snapshot are scanned with their live state) instead of streaming every
 * host per task; 0 disables it. Default 65536. Results are identical either way. Replaces the
 * per-task host scan of scheduler/vbp.py:43-47. */
int  pvt_set_band(pvt_ctx* ctx, int32_t min_hosts);
/* Window pipelining (default on): score window k+1 on a side stream while window k is walked.
 * Results are identical either way; off runs windows strictly one after the other. */
int  pvt_set_pipeline(pvt_ctx* ctx, int on);
/*
 * Group-parallel epochs (default on): a cost_aware best-fit round of several groups walks
 * consecutive groups of distinct anchor zones side by side, each on the epoch's start state,
 * and keeps exactly the prefix the sequential order would have produced (a group is rejected,
 * and walked again in the next epoch, if a host an earlier group committed to is its winner or
 * beats it); results are identical either way. Replaces the group loop of
 * scheduler/cost_aware.py:37-42 around _best_fit (:63-97).
 * pvt_epoch_stats: epochs run, segments walked and segments rejected in the last pvt_place.
 */
int  pvt_set_epochs(pvt_ctx* ctx, int on);
int  pvt_epoch_stats(pvt_ctx* ctx, int64_t* epochs, int64_t* segments, int64_t* rejected);
/*
 * Zero-cost frontier walk (default on; results identical either way): an epoch chain whose
 * tasks all find a zero-egress-cost host (score exactly 0) among the first 1024 hosts of its
 * zones is walked as a first fit over those hosts in LDS, with no candidate lists; the walk
 * proves each winner exact (pvt_zwalk.hip) and leaves any chain it cannot prove to the
 * list-based walk. pvt_zero_walk_stats: chains of the last pvt_place walked each way, and the
 * tasks of each epoch's longest chain (summed over its epochs: the walks' critical path).
 */
int  pvt_set_zero_walk(pvt_ctx* ctx, int on);
int  pvt_zero_walk_stats(pvt_ctx* ctx, int64_t* frontier_chains, int64_t* list_chains,
                         int64_t* longest_chain);
/* Counters of the last pvt_place call: windows run and refills forced by exhausted lists. */
int  pvt_last_stats(pvt_ctx* ctx, int64_t* windows, int64_t* refills);
/*
 * Host-dimension sharding (BASELINE config 5): `world` ranks (one per GPU)
 * each score a contiguous host range [host_lo, host_hi) and exchange per-task candidate
 * packages once per window; every rank then runs the same commit walk, so placements are
 * identical on all ranks and equal to pvt_place(). Each rank keeps the FULL availability array
 * (32 B per host, replicated and updated identically by the walk); only scoring is split.
 * The exchange is the caller's (an all-gather, e.g. RCCL through torch.distributed):
 *
 *   pvt_shard_begin(ctx, r, lo, hi, world, &max_bytes)     allocate send [max_bytes] and
 *                                                          recv [world * max_bytes] (device)
 *   loop:
 *     pvt_shard_score(ctx, send, &nt, &bytes)              nt == 0: the round is done
 *     all-gather `bytes` from every rank into recv, rank order, contiguous (recv[k*bytes..])
 *     pvt_shard_commit(ctx, recv)                          PVT_ESTALE: score again
 *
 * pvt_shard_commit launches the window's commit walk and returns without waiting for it
 * (pvt_set_pipeline on, the default): the next pvt_shard_score scores the following window on
 * a side stream while the walk runs and returns its package (complete on return), so the
 * caller's exchange -- issued on a stream that does not wait for the context's stream -- also
 * overlaps the walk. If that walk stops early the speculative package is stale: the next
 * pvt_shard_commit returns PVT_ESTALE on every rank and the caller scores again. With the
 * pipeline off every call completes its window before returning.
 * Opportunistic rounds shard by whole super-chunks of 16384 hosts: rank r of world W must take
 * hosts [r * P * 16384, (r + 1) * P * 16384) clamped to H, P = ceil(ceil(H / 16384) / W); the
 * packages carry its per-task feasibility bitmaps and super-chunk counts and every rank runs the
 * same draw / selection walk (windows of 256 tasks, not pipelined).
 *
 * `r` and its arrays must stay valid until the round is done. nt and bytes are the same on
 * every rank (window sizes depend only on walk results, which every rank shares).
 * Replaces the per-task scan of scheduler/cost_aware.py:88-92,
 * :118-122 and scheduler/vbp.py:19-22, :43-47 over a cluster too large for one GPU's pass.
 */
#define PVT_SHARD_MAX_WORLD 64
int  pvt_shard_begin(pvt_ctx* ctx, const pvt_round* r, int32_t host_lo, int32_t host_hi,
                     int32_t world, int64_t* max_package_bytes);
int  pvt_shard_score(pvt_ctx* ctx, void* package, int32_t* n_tasks, int64_t* package_bytes);
int  pvt_shard_commit(pvt_ctx* ctx, const void* packages);
/*
 * Resident rounds and scenario batches (BASELINE configs 1, 2 and 4; SURVEY.md §8(e), §8(f)
 * rank 2). A round with n_hosts <= PVT_RESIDENT_MAX_HOSTS and n_tasks <= PVT_RESIDENT_MAX_TASKS
 * fits one workgroup: its hosts stay in registers for the whole round and every task rescans
 * them (the reference's loop, restated). pvt_place_batch() runs n such rounds of ONE policy
 * (rounds[i].mode all equal) in a single launch, one workgroup per round, so independent
 * scenarios' rounds run side by side on all CUs. `rounds` is a HOST array of descriptors whose
 * array pointers are device pointers, exactly as for pvt_place() (mt_state in host memory);
 * each round is placed exactly as pvt_place() would place it. Synchronises before returning.
 * Returns PVT_EUNSUPPORTED if a round exceeds the limits (use pvt_place for it).
 *
 * pvt_set_resident(ctx, max_hosts): pvt_place() runs rounds with n_hosts <= max_hosts (and
 * n_tasks within the limit) as a batch of one; 0 disables it (the windowed score/commit path
 * runs every round). Default PVT_RESIDENT_MAX_HOSTS. Results are identical either way.
 */
#define PVT_RESIDENT_MAX_HOSTS 4096
#define PVT_RESIDENT_MAX_TASKS 4096
int  pvt_place_batch(pvt_ctx* ctx, const pvt_round* rounds, int32_t n_rounds);
/* pvt_place_batch with the rounds' MT19937 states resident on the device: mt_dev[n_rounds][625]
 * (in/out, key then pos, as mt_state), so no state crosses PCIe; the rounds' mt_state fields are
 * ignored. The scenario-batch driver (config 4) keeps its states on the device across rounds. */
int  pvt_place_batch_mt(pvt_ctx* ctx, const pvt_round* rounds, int32_t n_rounds, uint32_t* mt_dev);
int  pvt_set_resident(pvt_ctx* ctx, int32_t max_hosts);
/*
 * Anchor resolution for cost_aware groups (replaces the Counter/max of
 * CostAwareGlobalScheduler._group_tasks, scheduler/cost_aware.py:45-58).
 *
 * Item c (a container of ready tasks) has the predecessor list list[off[c] .. off[c+1]): the
 * placement of every task of every predecessor container, in the reference's iteration order
 * (app.get_predecessors(c.id) order = the container's `dependencies` order, application/
 * __init__.py:87-92,137-139; then p.tasks order). An entry is a host index (-1 = a predecessor
 * task without placement), or, when inst_host is set, an index into inst_host (a per-instance
 * host table kept resident in HBM, e.g. pivot_place.trace.DeviceTrace).
 * Outputs per item: mode_host = the host with the highest count, the first seen among equal
 * counts (Counter insertion order + max's first maximum); anchor_zone = zone[mode_host], or
 *   -1  empty list (the task groups by its application, cost_aware.py:56-57),
 *   -2  the mode entry is -1 (the reference raises AttributeError on get_host(None).locality),
 *   -3  invalid row, offsets or index out of range (the call then returns PVT_EINVAL).
 * With `item` set, item c uses row item[c] of a resident list table instead: its list is
 * list[off[item[c]] .. off[item[c]+1]) (off then has n_rows + 1 entries), so a trace kept in
 * HBM uploads only the ready containers' row numbers per round.
 * All pointers are device pointers. Lists may hold up to 2^30 entries. Synchronises before
 * returning.
 */
typedef struct pvt_anchor_args {
  int32_t n_items;            /* C                                                        */
  int32_t n_hosts;            /* H                                                        */
  int64_t n_pred;             /* length of list                                           */
  int64_t n_inst;             /* length of inst_host (0 when inst_host is NULL)           */
  const int64_t* off;         /* [C+1], or [n_rows+1] when item is set                    */
  const int32_t* list;        /* [n_pred]                                                 */
  const int32_t* inst_host;   /* [n_inst] or NULL                                         */
  const int32_t* zone;        /* [H]                                                      */
  int32_t* mode_host;         /* [C] out                                                  */
  int32_t* anchor_zone;       /* [C] out                                                  */
  const int32_t* item;        /* [C] row of off per item, or NULL (item c = row c)        */
  int64_t n_rows;             /* rows of off when item is set (0 when item is NULL)       */
} pvt_anchor_args;
int  pvt_anchor(pvt_ctx* ctx, const pvt_anchor_args* a);

/*
 * Drop-in round from HOST memory in one round trip (the reference's synchronous schedule()
 * call, scheduler/__init__.py:100-103). Every array pointer of r is a HOST pointer: avail
 * in/out, placement and order out, mt_state in/out. The context packs the inputs into its
 * pinned staging buffer, copies them to the device with ONE copy, places the round, and copies
 * avail, placement, order and the MT19937 states back with ONE copy and one synchronisation.
 * On error the outputs are left untouched.
 *
 * cost_aware rounds may pass `items` and leave task_group / group_anchor NULL: the grouping of
 * scheduler/cost_aware.py:30-58 then runs on the device in the same round trip -- per item the
 * mode host of its predecessor placements (as pvt_anchor), groups keyed by the storage of that
 * host's zone or, for items without predecessors, by their application, numbered in first-seen
 * task order, and one randomizer.choice(storage) per application group, in group order, from
 * items->mt_state (the policy's RandomState; in/out). items->status[0] returns the number of
 * groups, status[1] an error kind with PVT_EINVAL: 1 a mode placement that is not a host of the
 * cluster, 2 a zone without storage (the reference raises AttributeError for both), 3 malformed
 * item lists. Rounds beyond the fused grouping's limits (T > 16384, n_storage + n_apps > 8192)
 * return PVT_EUNSUPPORTED before any work (the caller then uses pvt_anchor + pvt_place).
 */
typedef struct pvt_ca_items {
  int32_t n_items;             /* C: distinct containers of the ready tasks                 */
  int32_t n_apps;              /* applications of the items (item_app in [0, n_apps))        */
  int64_t n_pred;              /* length of pred_host                                       */
  const int32_t* task_item;    /* [T] item of each task                                     */
  const int64_t* pred_off;     /* [C+1] item c's predecessor placements pred_off[c..c+1)     */
  const int32_t* pred_host;    /* [n_pred] host index of each placement, -1 = not a host     */
  const int32_t* item_app;     /* [C] application of each item                               */
  int32_t n_storage;           /* S = len(cluster.storage)                                   */
  int32_t reserved;            /* must be 0                                                  */
  const int32_t* storage_zone; /* [S] zone of each storage, cluster.storage order            */
  const int32_t* zone_storage; /* [Z] storage index of get_storage_by_locality(zone), -1 None */
  uint32_t* mt_state;          /* [625] in/out: the policy randomizer (MT19937 key + pos)    */
  int32_t* status;             /* [2] out: groups formed, error kind                         */
} pvt_ca_items;
int  pvt_place_host(pvt_ctx* ctx, pvt_round* r, pvt_ca_items* items);
/*
 * Several independent drop-in rounds from HOST memory in one round trip: the lock-step driver's
 * tick, where simulations running different policies each wait on one schedule() round
 * (scheduler/__init__.py:100-103 once per simulation). rounds[i] is as for pvt_place_host, with
 * items[i] its optional fused cost_aware grouping (items itself may be NULL); the policies may
 * differ between rounds. Every round with tasks must fit the resident limits (n_hosts <=
 * min(pvt_set_resident limit, PVT_RESIDENT_MAX_HOSTS), n_tasks <= PVT_RESIDENT_MAX_TASKS) --
 * else PVT_EUNSUPPORTED before any work. One staging copy up, one launch for all rounds (one
 * workgroup each), one copy back, one synchronisation. rcs[i] receives each round's own result
 * (PVT_OK, or PVT_EINVAL with items[i]->status[1] set for a grouping error, its outputs then
 * untouched); the call returns PVT_OK when the batch ran.
 */
int  pvt_place_host_batch(pvt_ctx* ctx, pvt_round* rounds, pvt_ca_items* const* items,
                          int32_t n_rounds, int32_t* rcs);

/*
 * Replay support (no reference counterpart): avail[r][h] = avail0[r][h], r = 0..3, for every
 * h = hosts[i], i < n, with 0 <= h < n_hosts (other entries are ignored), on the context's
 * stream; device pointers. A round placed again from the same snapshot needs only the hosts
 * its placement names restored -- a round changes no other capacity -- so passing the round's
 * placement array as `hosts` resets it in one small launch instead of a copy of all 4 x H.
 */
int  pvt_restore_hosts(pvt_ctx* ctx, double* avail, const double* avail0, int32_t n_hosts,
                       const int32_t* hosts, int32_t n);

/*
 * Meter aggregates of a batch of S scenarios (replaces the properties
 * Meter.cumulative_instance_hours, .total_network_traffic_cost and .average_congestion_delay,
 * resources/meter.py:31-53, read by alibaba/runner.py:45-51 via Meter.save).
 *
 * The logs are nested CSR arrays in the meter's own dict orders:
 *   scenario s -> hosts  host_off[s] .. host_off[s+1]          (Meter.__hosts)
 *   host h     -> intervals iv_off[h] .. iv_off[h+1]: [iv_start, iv_end] (check-in/out)
 *   scenario s -> routes route_off[s] .. route_off[s+1]        (Meter.__routes)
 *   route r    -> packets pkt_off[r] .. pkt_off[r+1]; route_cost[r] = cost[src.loc, dst.loc]
 *   packet p   -> transfers tr_off[p] .. tr_off[p+1]: [tr_start, tr_end, tr_size]
 * Per scenario: instance_hours = sum_h sum_v (end - start) / 3600; egress_cost = sum_r
 * route_cost * (sum_p sum_t size) / 8000 (ResourceMetadata.calc_network_traffic_cost,
 * resources/__init__.py:565-569); congestion_delay = sum over consecutive transfers of a packet
 * of (start_i - end_{i-1}) / #packets, 0 without packets. Per host and per route the sums run
 * in the reference's order; across hosts / routes a fixed tree (fp64, within 1e-9 relative of
 * the reference's left-to-right sum). All pointers are device pointers. Returns PVT_EINVAL if an
 * offset is out of range. Synchronises before returning.
 */
typedef struct pvt_meter_log {
  int32_t n_scen;             /* S                                                        */
  int32_t reserved;           /* must be 0                                                */
  int64_t n_host_rows, n_iv, n_routes, n_pkts, n_tr;   /* lengths of the level arrays    */
  const int64_t* host_off;    /* [S+1]                                                    */
  const int64_t* iv_off;      /* [n_host_rows+1]                                          */
  const double* iv_start;     /* [n_iv]                                                   */
  const double* iv_end;       /* [n_iv]                                                   */
  const int64_t* route_off;   /* [S+1]                                                    */
  const double* route_cost;   /* [n_routes]                                               */
  const int64_t* pkt_off;     /* [n_routes+1]                                             */
  const int64_t* tr_off;      /* [n_pkts+1]                                               */
  const double* tr_start;     /* [n_tr]                                                   */
  const double* tr_end;       /* [n_tr]                                                   */
  const double* tr_size;      /* [n_tr]                                                   */
  double* instance_hours;     /* [S] out                                                  */
  double* egress_cost;        /* [S] out                                                  */
  double* congestion_delay;   /* [S] out                                                  */
} pvt_meter_log;
int  pvt_meter(pvt_ctx* ctx, const pvt_meter_log* m);

/* Human-readable text of the last error on this context (static storage of the ctx). */
const char* pvt_last_error(pvt_ctx* ctx);

#ifdef __cplusplus
}
#endif

#endif /* PIVOT_PLACE_H */
