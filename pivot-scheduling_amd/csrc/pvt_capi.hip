// pvt_capi.hip — the C ABI (include/pivot_place.h): context, scratch and the per-round driver.
//
// pvt_place() replaces the body of a reference policy's schedule() (scheduler/__init__.py:79-80,
// called at :103). A round runs as:
//   1. a2 order: tasks grouped (cost_aware groups, cost_aware.py:37) and stably sorted by
//      descending ||d||2 (cost_aware.py:60-61, vbp.py:17,41) with two stable radix sorts.
//   2. windows of up to W tasks: candidate lists for the window on the current state (score +
//      merge kernels, or the ordered scan for index-order first-fit), then the commit walk. A
//      walk that meets an exhausted list stops early; the next window starts at that task.
//   3. cost_aware first-fit with sort_hosts recomputes the frozen host key at every group start
//      (cost_aware.py:118-119), so its windows never cross a group boundary.
// Opportunistic (PVT_OPP) runs its own count/select kernels (pvt_opp.hip).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <limits>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "pivot_place.h"
#include "pvt_kernels.h"
#include "pvt_opp.h"
#include "pvt_anchor.h"
#include "pvt_groups.h"
#include "pvt_meter.h"

using namespace pvt;

// Group-parallel epochs (cost_aware best-fit): at most EPOCH_SEGS group segments, walked in at
// most EPOCH_SEGS chains of <= CHAIN_MAX tasks, and EPOCH_MAX tasks per epoch (its lists: 64 B
// x LMAX per task).
static constexpr int EPOCH_SEGS = 64;
static constexpr int EPOCH_MAX = 16384;
// ep_dev / ep_host words: uploaded [seg_off | seg_chain | seg_cstart | coff | csoff | cseg |
// cmap], then read back [status (2 per chain) | bad (per segment)]
static constexpr int EP_SEG_OFF = 0, EP_SEG_CHAIN = EP_SEG_OFF + EPOCH_SEGS + 1,
                     EP_SEG_CSTART = EP_SEG_CHAIN + EPOCH_SEGS, EP_COFF = EP_SEG_CSTART + EPOCH_SEGS,
                     EP_CSOFF = EP_COFF + EPOCH_SEGS + 1, EP_CSEG = EP_CSOFF + EPOCH_SEGS + 1,
                     EP_CMAP = EP_CSEG + EPOCH_SEGS, EP_STATUS = EP_CMAP + EPOCH_MAX,
                     EP_BAD = EP_STATUS + 2 * EPOCH_SEGS, EP_RES = EP_BAD + EPOCH_SEGS,
                     EP_SAFE = EP_RES + 8;
static constexpr int EP_WORDS = EP_SAFE + EPOCH_SEGS;
static constexpr int KEYED_FRONTIER_MIN = 32;   // group tasks worth a frontier-walk launch
static constexpr int ORDERED_FRONTIER_MIN = 32;  // tasks a frontier attempt must place to go on
static constexpr int AHEAD_MAX = 8;             // vbp best-fit walks enqueued per host round trip
static constexpr int ORDERED_FRONTIER_TASKS = 4096;   // tasks per frontier attempt (default;
                                                       // config-5 vbp_ff sweep: 512 1.75, 1024
                                                       // 1.09, 2048 0.94, 4096 0.90, 8192 0.98 ms)
static constexpr int ORDERED_FRONTIER_HOSTS = 65536;   // first span of hosts the window is taken from
// vbp best-fit: candidate lists by a memory band over hosts sorted once per round (pvt_band.hip)
// from this many hosts (per shard) on, with this many list segments per task
static constexpr int BAND_MIN_HOSTS = 65536;
static constexpr int BAND_SEGS = 16;

struct Buf {
  void* p = nullptr;
  size_t n = 0;
};

struct TimedLaunch {
  int kclass;
  const char* kname;   // the one kernel the scope brackets (pvt_get_kernel_kstats), or NULL
  double candidates, bytes;
  hipEvent_t a, b;
};

// The next epoch from task t0: consecutive group segments (processing order), each assigned to
// the chain of its anchor's zero-cost component (two groups of one component compete for the
// same hosts: one walk takes them in order). A chain holds at most CHAIN_MAX tasks; a segment
// that ends inside its group ends the epoch (the rest of the group depends on it).
struct EpochPlan {
  std::vector<int> off, chain, cstart;     // segments: window offsets (+ end), chain, start in it
  std::vector<std::vector<int>> segs;      // chains: their segments
  std::vector<int> len;                    // chains: tasks
};

// Package kinds of a host-sharded round (pvt_shard_*): candidate lists of a window, or the
// window candidates of a frontier walk (FrontierHdr + FrontierSlot per chain / walk).
enum { PK_LIST = 0, PK_EPOCH = 1, PK_KEYED = 2, PK_ORDERED = 3 };

struct RoundState {
  pvt_round r;                    // the caller's round (arrays stay caller-owned)
  bool active = false;
  int T = 0, H = 0, Z = 0, lo = 0, hi = 0, world = 0;
  bool keyed = false, ordered = false;
  bool kscan = false;             // keyed first-fit lists from the per-group sorted order
  int kmode = 0;                  // 1: zero-key prefix in host order, 2: full sort
  int kn = 0;                     // hosts in the current order (prefix length in mode 1)
  bool kstall = false;            // a walk found a prefix list exhausted: sort the rest
  int32_t* ord = nullptr;         // processing order (ctx scratch)
  std::vector<int> gstart, ganchor, gid;   // keyed groups: starts, anchors, caller's group ids
  size_t g = 0, ngroups = 0;
  int key_group = -1;             // group whose frozen first-fit key is computed
  int t0 = 0, W = 0, Wmax = 0, nt = 0;
  int lb = 0;                     // list buffer of the current window
  // host-sharded opportunistic rounds: windows of opp_W tasks; this rank counts super-chunks
  // [opp_sq_lo, opp_sq_hi); packages hold opp_Psq super-chunks per task (the largest share)
  bool opp = false;
  int opp_W = 0, opp_nq = 0, opp_nsq = 0, opp_Psq = 0, opp_sq_lo = 0, opp_sq_hi = 0;
  // host-sharded list rounds, pipelined: the walk in flight (window if_t0 + [0, if_nt) on list
  // buffer if_lb) and the scored window awaiting its exchange (pt0, nt, plb; spec = scored
  // while a walk was in flight, so it inherits that walk's hosts)
  bool inflight = false, spec = false, if_inh = false;   // if_inh: the walk in flight
  int if_t0 = 0, if_nt = 0, if_lb = 0, pt0 = 0, plb = 0;   //   inherited touched hosts
  std::vector<int> egs, ega;      // cost_aware best-fit epochs: group starts (+ T) and anchors
  std::vector<int> ecomp;         // zone -> its component of zones joined by zero egress cost
  bool in_epoch = false;          // lists scored for an epoch (place_epochs)
  bool ofront = false;            // ordered first-fit rounds walked by the frontier walk
  int ofh = 0;                    // hosts the frontier window is taken from
  // grouped rounds: per-group task counts, group anchors and (cost_aware) the cost table,
  // copied to the host once by build_order (one synchronisation) for the group plans
  bool ginfo = false;
  std::vector<int32_t> gcnt, ga_host;
  std::vector<double> cost_host;
  int of_tasks = ORDERED_FRONTIER_TASKS;   // tasks per ordered frontier attempt
  // host-sharded rounds (pvt_shard_*) on the frontier walks: the scored package's kind and size,
  // and what comes next
  bool sharded = false;
  int pkind = PK_LIST;
  int64_t pbytes = 0;
  bool sh_epochs = false;         // cost_aware best-fit: frontier epochs between list windows
  int list_until = 0;             //   list windows up to this task (a chain left unproven), then
                                  //   epochs again
  EpochPlan E;                    //   the epoch of the scored package
  bool of_try = false;            // ordered rounds: a frontier attempt comes next
  int of_n = 0, of_hs = 0;        //   the scored attempt's tasks and host span
  bool kf_pending = false;        // keyed rounds: the group start's frontier walk comes next
  bool ffe = false;               // keyed rounds: first-fit zero-key epochs (ff_epoch)
  bool hmin_pre = false;          // the first epoch's host minima were queued by round_begin
  bool zpre = false;              // ... and its zero-cost windows were prebuilt (ctx->zwin)
  bool stage_flag = false;        // the grouped order's counts are signalled by ctx->flag_host
  bool gathered = false;          // ... and group_sort_gather_kernel wrote the gathered order
  bool prep_fused = false;        // build_order's order_scatter_kernel filled placement / zone tables
  int ffe_skip = -1;              //   the group they could not start (the keyed path takes it)
  // vbp best-fit band lists (pvt_band.hip): the sorted snapshot of hosts [lo, hi) is built; a
  // walk whose committed hosts are not yet flagged as touched (its own-ids buffer)
  bool band = false;
  int band_S = BAND_SEGS;
  int touch_lb = -1;
  const int32_t* touch_status = nullptr;   //   (its status: [1] = hosts in the own-ids buffer)
  bool reps[2] = {false, false};  //   list buffer b holds representative rows (the round's runs)
  int rbase[2] = {0, 0};          //     the run of its window's first task
  std::vector<int32_t> runs;      //   the round's run ids (band_runs_kernel), on the host
  bool full_lists = false;        //   (one list per task: the list walk's fallback)
  bool lw_last = false;           // the walk in flight is the one-wave list walk (pvt_lwalk.hip)
  bool lw_flag = false;           //   reporting through ctx->flag_host[4..6] (no copy, no sync)
  int lw_lb = 0, lw_prev = 0;     //   its list buffer and inherited hosts (for the fallback)
};

struct pvt_ctx {
  int device = 0;
  hipStream_t own = nullptr, stream = nullptr;
  hipStream_t side = nullptr;     // scores the next window while the current one is walked
  hipEvent_t ev_lists = nullptr;   // side stream: the next window's lists are ready
  hipEvent_t ev_walk = nullptr;    // caller stream: everything before the current walk is done
  hipEvent_t ev_stage = nullptr;   // the grouped order's counts are in the pinned stage
  int walk_cus = 0;                // CUs the side stream leaves to the walks
  std::string err;
  int window = 0;                 // 0: per-policy default
  int64_t windows = 0, refills = 0;
  int profiling = 0;               // 0 off, 1 every launch, 2 the named kernels only
  std::string prof_only;           //   (2: this one named kernel, when set)
  int bind_events = 1;             //   (2: events bound to the kernel's dispatch; PVT_BIND_EVENTS)
  int64_t n_unbound = 0;           //   (2: named scopes whose bound events were dropped)
  pvt_kstats ks[PVT_K_COUNT];
  std::vector<hipEvent_t> evpool;
  std::vector<TimedLaunch> pending;
  std::map<std::string, pvt_kstats> kks;   // per kernel (scopes tagged with its name)
  // scratch
  Buf gcnt, goff, gskey, gsidx;   // grouped order: counts, offsets + cursors, scattered pairs
  Buf ord, ord2, keys64a, keys64b, keys32a, keys32b, sorttmp, dem_ord, anc_ord, grp_ord, csum, bsum, key,
      seg, seg_feas, l_e[2], l_ids[2], l_t[2], next, opp, pkg, owned[2], rdesc, rmt, anc_scr, oppfault, kskey, kperm, kiota, ksorttmp, kflag;
  int pipeline = 1;               // overlap scoring of window k+1 with the walk of window k
  int keyed_scan = 1;             // keyed first-fit: sorted host order + early-exit scan
  int score_tw = 0;               // score kernel tasks per wave (0: policy default; 2 or 4)
  int resident_max = PVT_RESIDENT_MAX_HOSTS;   // pvt_place: resident kernel up to this many hosts
  int epochs = 1;                 // cost_aware best-fit: group-parallel speculative epochs
  int64_t n_epochs = 0, n_segs = 0, n_rejected = 0;
  int64_t n_zchains = 0, n_gchains = 0;   // epoch chains walked by the frontier / list walk
  int64_t n_longest = 0;                  // tasks of the longest epoch chain (sum over epochs)
  int zwalk = 1;                          // zero-cost frontier walk of epoch chains
  int of_tasks = ORDERED_FRONTIER_TASKS;  // ordered frontier tasks per attempt (PVT_OF_TASKS)
  Buf fwin;                               // host-sharded frontier walks: merged windows
  int band_min = BAND_MIN_HOSTS;          // vbp best-fit band lists from this many hosts (0: off)
  int lwalk = 1;                          // vbp best-fit windows: the one-wave list walk
  // tuning / A-B knobs, read from the environment once, at pvt_ctx_create (never per round):
  int t_segments = 0;             // PVT_SEGMENTS: score-pass host segments (0: by policy)
  int t_band_segs = 0;            // PVT_BAND_SEGS: vbp best-fit band list segments (0: default)
  int t_keyed_scan = -1;          // PVT_KEYED_SCAN: keyed first-fit scan on / off (-1: keyed_scan)
  int t_of_hosts = 0;             // PVT_OF_HOSTS: ordered frontier host span (0: default)
  int t_epoch_plan = 1;           // PVT_EPOCH_PLAN: 0 = epoch chains by distinct zone only
  int t_zpre = 1;                 // PVT_ZPRE: 0 = every frontier walk builds its own window
  int t_chain_tab = 1;            // PVT_CHAIN_TAB: 0 = chain tables uploaded before the walk
  int t_merge_bitonic = 0;        // PVT_MERGE_SMALL=0: the bitonic merge always
  int res_waves = 4;              // PVT_RES_WAVES: waves per resident round (2, 4 or 8)
  int rwalk = 9;                  // PVT_RWALK: resident one-wave walks, bits 1 cost_aware best-fit, 8
                                  //   first fit by index, 4 without bulk runs, 2 rotated walker; 0 none;
                                  //   4-wave path: 16 no bulk sticky runs, 32 no run lists, 64 run lists
                                  //   for every policy, bits 8-15 the shortest remaining run given a list (A/B)
  int fused = 1;                  // PVT_FUSED=0: host batches staged in six launches (A/B)
  int ahead = 0;                  // PVT_AHEAD=1: vbp best-fit walks enqueued ahead (place_ahead;
                                  // measured slower, kept for A/B)
  Buf wslot;                      // enqueued-ahead walks' status slots (place_ahead)
  Buf bkey, bidx, bsa, bstb, btouch, btlist, btcnt, bsorttmp;   // band lists: sorted snapshot
  Buf brec;                       // band lists: the snapshot's host records (BandRec)
  Buf bpos, bptouch;              // band lists: host -> sorted position, touched by position
  Buf brun, brdem;                // band lists: the round's runs of equal demands (ids, demands)
  Buf ep_dev, wres;               // epoch tables / status / flags, per-task commit logs
  Buf hmin;                       // frontier walk: per-dimension host minima (partials)
  Buf cmax;                       // frontier-walked epochs: chains' largest demands
  Buf zwin;                       // the first epoch's zero-cost windows (ZoneWindows)
  int32_t* ep_host = nullptr;     // pinned staging of ep_dev
  int32_t* ep_hdev = nullptr;     // ep_host's device address (the accept kernel's readback)
  pvt_round* rstage = nullptr;    // pvt_place_batch: descriptors staged for the device (pinned)
  size_t rstage_cap = 0;
  hipEvent_t ev_rstage = nullptr;  //   recorded after their upload (and the MT states')
  bool rstage_busy = false;
  uint32_t* rmt_host = nullptr;   //   and the rounds' MT19937 states (pinned)
  size_t rmt_cap = 0;
  RoundState rs;
  int32_t* next_host = nullptr;   // pinned
  int32_t* flag_host = nullptr;   // pinned word the grouped order's count kernel stores to
  int32_t* flag_hdev = nullptr;   //   (its device address)
  int32_t flag_seq = 0;
  int32_t walk_seq = 0;           // the one-wave list walk's report in flag_host[4..6]
  void* gstage = nullptr;         // grouped order: counts, anchors, cost table (pinned)
  size_t gstage_cap = 0;
  uint64_t* stamps = nullptr;     // PVT_STAMPS builds: device per-phase cycle sums
  void* hst = nullptr;            // pvt_place_host: pinned staging of a host-memory round
  void* hst_map = nullptr;        //   (its device address: the copy kernels' side)
  size_t hst_cap = 0;
  Buf hdev;                       //   and its device copy
  // the zone tables of the last host-array round (cost then bw, Z x Z each) kept on the device:
  // drop-in rounds of one cluster pass the same tables every time, so they are not staged again
  std::vector<double> zt_host;
  Buf zt_dev;
  int zt_Z = 0;
};

static int fail(pvt_ctx* c, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return code;
}

#define HIPCHK(expr)                                                                     \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess)                                                                \
      return fail(ctx, PVT_EHIP, "%s failed: %s", #expr, hipGetErrorString(e_));         \
  } while (0)

static int ensure(pvt_ctx* ctx, Buf& b, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (b.n >= bytes) return PVT_OK;
  const size_t want = std::max(bytes, b.n * 3 / 2);
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.n = 0;
  if (hipMalloc(&b.p, want) != hipSuccess) {
    b.p = nullptr;
    return fail(ctx, PVT_ENOMEM, "hipMalloc(%zu) failed", want);
  }
  b.n = want;
  return PVT_OK;
}
#define ENSURE(b, bytes)                              \
  do {                                                \
    int rc_ = ensure(ctx, (b), (bytes));              \
    if (rc_) return rc_;                              \
  } while (0)

template <class T>
static T* P(Buf& b) { return reinterpret_cast<T*>(b.p); }

// ---------------------------------------------------------------- profiling
// Timing-only events: no system-scope fence when they complete (no cache writeback and
// invalidate between the timed kernel and its neighbours; the marker of a default event cost
// ~5 us of idle GPU per record on the default line).
static constexpr unsigned PROFILE_EVENT_FLAGS = hipEventDisableSystemFence;
static hipEvent_t take_event(pvt_ctx* ctx) {
  if (!ctx->evpool.empty()) {
    hipEvent_t e = ctx->evpool.back();
    ctx->evpool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreateWithFlags(&e, PROFILE_EVENT_FLAGS);
  return e;
}
namespace pvt { thread_local TimedEvents g_timed; }
// A profiling scope. profiling 1: events recorded around the scope's launches. profiling 2 (one
// named kernel): the events are bound to that kernel's dispatch by PVT_LAUNCH (pvt_kernels.h),
// with no marker packets in the stream; PVT_BIND_EVENTS=0 records them around it instead.
struct Scope {
  pvt_ctx* ctx;
  hipStream_t st;
  TimedLaunch t;
  bool bound = false;
  Scope(pvt_ctx* c, int kclass, double cand, double bytes, hipStream_t s = nullptr,
        const char* kname = nullptr)
      : ctx(c), st(s ? s : c->stream) {
    t.kclass = kclass; t.kname = kname; t.candidates = cand; t.bytes = bytes; t.a = t.b = nullptr;
    if (!on()) return;
    t.a = take_event(ctx);
    if (ctx->profiling == 2 && ctx->bind_events && !g_timed.armed) {
      t.b = take_event(ctx);
      g_timed.a = t.a; g_timed.b = t.b; g_timed.armed = true; g_timed.used = g_timed.extra = 0;
      bound = true;
    } else {
      (void)hipEventRecord(t.a, st);
    }
  }
  bool on() const {
    return ctx->profiling == 1 ||
           (ctx->profiling == 2 && t.kname && (ctx->prof_only.empty() || ctx->prof_only == t.kname));
  }
  ~Scope() {
    if (!on()) return;
    if (bound) {
      const bool ok = g_timed.used == 1 && g_timed.extra == 0;
      g_timed = TimedEvents{};
      if (ok) {
        ctx->pending.push_back(t);
      } else {                        // no launch, or more than the one the events bound to
        ctx->evpool.push_back(t.a);
        ctx->evpool.push_back(t.b);
        ctx->n_unbound++;
      }
      return;
    }
    t.b = take_event(ctx);
    (void)hipEventRecord(t.b, st);
    ctx->pending.push_back(t);
  }
};
static void harvest(pvt_ctx* ctx) {
  for (auto& t : ctx->pending) {
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, t.a, t.b);
    pvt_kstats& k = ctx->ks[t.kclass];
    k.launches += 1; k.ms += ms; k.candidates += t.candidates; k.bytes += t.bytes;
    if (t.kname) {
      pvt_kstats& n = ctx->kks[t.kname];
      n.launches += 1; n.ms += ms; n.candidates += t.candidates; n.bytes += t.bytes;
    }
    ctx->evpool.push_back(t.a);
    ctx->evpool.push_back(t.b);
  }
  ctx->pending.clear();
}

// ---------------------------------------------------------------- ABI
extern "C" int pvt_abi_version(void) { return PVT_ABI_VERSION; }

// The side stream (the next window's score / count pass while a walk runs) is ordered against
// the walks by events only -- no in-kernel flag polled by the command processor, which never
// completes under serialising tools (rocprofv3 counter collection) -- and runs at the lowest
// queue priority (the context's own stream at the highest), so when walk k and the side pass k+1 become ready together (walk k-1 done)
// the walk, one workgroup that needs a whole CU's LDS, is dispatched first. PVT_WALK_CUS=n keeps
// the side stream off n CUs instead (measured: it serialises the two streams).
static hipError_t create_streams(pvt_ctx* ctx, int ncu) {
  int prio = 1;
  if (const char* e = getenv("PVT_SIDE_PRIO")) prio = atoi(e);
  int least = 0, greatest = 0;
  if (prio && (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess || least == greatest))
    prio = 0;
  hipError_t e = prio ? hipStreamCreateWithPriority(&ctx->own, hipStreamNonBlocking, greatest)
                      : hipStreamCreateWithFlags(&ctx->own, hipStreamNonBlocking);
  if (e != hipSuccess) return e;
  int cus = 0;
  if (const char* e = getenv("PVT_WALK_CUS")) cus = atoi(e);   // tuning experiments
  if (cus > 0 && ncu > 2 * cus) {
    std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
    const int stride = ncu / cus;
    int kept = 0;
    for (int i = 0; i < ncu; i++)
      if (i % stride != stride - 1 || i / stride >= cus) { mask[i / 32] |= 1u << (i % 32); kept++; }
    if (hipExtStreamCreateWithCUMask(&ctx->side, (uint32_t)mask.size(), mask.data()) == hipSuccess) {
      ctx->walk_cus = ncu - kept;
      return hipSuccess;
    }
    (void)hipGetLastError();
  }
  ctx->walk_cus = 0;
  if (prio) return hipStreamCreateWithPriority(&ctx->side, hipStreamNonBlocking, least);
  return hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking);
}

extern "C" int pvt_ctx_create(int device, pvt_ctx** out) {
  if (!out) return PVT_EINVAL;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= device || device < 0) return PVT_ENODEV;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return PVT_ENODEV;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return PVT_ENODEV;
  pvt_ctx* ctx = new pvt_ctx();
  ctx->device = device;
  std::memset(ctx->ks, 0, sizeof(ctx->ks));
  if (hipSetDevice(device) != hipSuccess ||
      create_streams(ctx, prop.multiProcessorCount) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_lists, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_walk, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_stage, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_rstage, hipEventDisableTiming) != hipSuccess ||
      init_kernel_attrs() != hipSuccess || pvt::opp_init_attrs() != hipSuccess ||
      resident_init_attrs() != hipSuccess || lwalk_init_attrs() != hipSuccess ||
      hipHostMalloc((void**)&ctx->next_host, sizeof(int32_t) * (4 + 4 * AHEAD_MAX)) != hipSuccess ||
      hipHostMalloc((void**)&ctx->flag_host, sizeof(int32_t) * 16, hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void**)&ctx->flag_hdev, ctx->flag_host, 0) != hipSuccess ||
      hipHostMalloc((void**)&ctx->ep_host, sizeof(int32_t) * EP_WORDS) != hipSuccess ||
      hipHostGetDevicePointer((void**)&ctx->ep_hdev, ctx->ep_host, 0) != hipSuccess) {
    delete ctx;
    return PVT_EHIP;
  }
  std::memset(ctx->flag_host, 0, sizeof(int32_t) * 16);   // (flag_seq starts at 0: no stale 1)
  ctx->stream = ctx->own;
  if (const char* e = getenv("PVT_OF_TASKS")) ctx->of_tasks = std::max(32, atoi(e));   // tuning
  if (const char* e = getenv("PVT_BAND")) ctx->band_min = std::max(0, atoi(e));       // A/B
  if (const char* e = getenv("PVT_LWALK")) ctx->lwalk = atoi(e) != 0;                  // A/B
  if (const char* e = getenv("PVT_AHEAD")) ctx->ahead = atoi(e) != 0;                  // A/B
  if (const char* e = getenv("PVT_RWALK")) ctx->rwalk = atoi(e);                       // A/B
  if (const char* e = getenv("PVT_FUSED")) ctx->fused = atoi(e) != 0;                  // A/B
  if (const char* e = getenv("PVT_BIND_EVENTS")) ctx->bind_events = atoi(e) != 0;      // A/B
  if (const char* e = getenv("PVT_SEGMENTS")) ctx->t_segments = std::max(1, atoi(e));  // tuning
  if (const char* e = getenv("PVT_BAND_SEGS")) ctx->t_band_segs = atoi(e);             // tuning
  if (const char* e = getenv("PVT_KEYED_SCAN")) ctx->t_keyed_scan = atoi(e) != 0;      // A/B
  if (const char* e = getenv("PVT_OF_HOSTS")) ctx->t_of_hosts = std::max(ZW_M, atoi(e));   // tuning
  if (const char* e = getenv("PVT_EPOCH_PLAN")) ctx->t_epoch_plan = atoi(e);           // A/B
  if (const char* e = getenv("PVT_ZPRE")) ctx->t_zpre = atoi(e) != 0;                  // A/B
  if (const char* e = getenv("PVT_CHAIN_TAB")) ctx->t_chain_tab = atoi(e) != 0;        // A/B
  if (const char* e = getenv("PVT_MERGE_SMALL")) ctx->t_merge_bitonic = atoi(e) == 0;  // A/B
  if (const char* e = getenv("PVT_RES_WAVES")) ctx->res_waves = atoi(e) == 8 ? 8 : atoi(e) == 2 ? 2 : atoi(e) == 1 ? 1 : 4;  // A/B
  *out = ctx;
  return PVT_OK;
}

extern "C" int pvt_ctx_destroy(pvt_ctx* ctx) {
  if (!ctx) return PVT_EINVAL;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  if (ctx->side) (void)hipStreamSynchronize(ctx->side);
  harvest(ctx);
  Buf* bufs[] = {&ctx->ord, &ctx->ord2, &ctx->keys64a, &ctx->keys64b, &ctx->keys32a, &ctx->keys32b,
                 &ctx->sorttmp, &ctx->dem_ord, &ctx->anc_ord, &ctx->grp_ord, &ctx->csum, &ctx->bsum, &ctx->key,
                 &ctx->seg, &ctx->seg_feas, &ctx->l_e[0], &ctx->l_ids[0], &ctx->l_t[0],
                 &ctx->l_e[1], &ctx->l_ids[1], &ctx->l_t[1], &ctx->next, &ctx->opp, &ctx->pkg,
                 &ctx->owned[0], &ctx->owned[1], &ctx->rdesc, &ctx->rmt, &ctx->anc_scr, &ctx->oppfault, &ctx->hdev, &ctx->kskey, &ctx->kperm, &ctx->kiota,
                 &ctx->ksorttmp, &ctx->kflag, &ctx->ep_dev, &ctx->wres, &ctx->hmin, &ctx->cmax, &ctx->fwin,
                 &ctx->bkey, &ctx->bidx, &ctx->bsa, &ctx->bstb, &ctx->btouch, &ctx->btlist,
                 &ctx->btcnt, &ctx->bsorttmp, &ctx->brun, &ctx->brdem, &ctx->bpos, &ctx->bptouch, &ctx->zt_dev,
                 &ctx->zwin, &ctx->brec};
  for (Buf* b : bufs)
    if (b->p) (void)hipFree(b->p);
  for (hipEvent_t e : ctx->evpool) (void)hipEventDestroy(e);
  if (ctx->next_host) (void)hipHostFree(ctx->next_host);
  if (ctx->flag_host) (void)hipHostFree(ctx->flag_host);
  if (ctx->ep_host) (void)hipHostFree(ctx->ep_host);
  if (ctx->gstage) (void)hipHostFree(ctx->gstage);
  if (ctx->hst) (void)hipHostFree(ctx->hst);
  if (ctx->rstage) (void)hipHostFree(ctx->rstage);
  if (ctx->rmt_host) (void)hipHostFree(ctx->rmt_host);
  if (ctx->ev_lists) (void)hipEventDestroy(ctx->ev_lists);
  if (ctx->ev_walk) (void)hipEventDestroy(ctx->ev_walk);
  if (ctx->ev_stage) (void)hipEventDestroy(ctx->ev_stage);
  if (ctx->ev_rstage) (void)hipEventDestroy(ctx->ev_rstage);
  if (ctx->side) (void)hipStreamDestroy(ctx->side);
  if (ctx->own) (void)hipStreamDestroy(ctx->own);
  delete ctx;
  return PVT_OK;
}

extern "C" int pvt_ctx_set_stream(pvt_ctx* ctx, void* stream) {
  if (!ctx) return PVT_EINVAL;
  ctx->stream = (hipStream_t)stream;   // NULL is the device's default (null) stream
  return PVT_OK;
}

// Events of the timed scopes come from a pool that harvest() refills; the pool is filled and
// every event recorded once when profiling is switched on, so a timed round neither creates an
// event nor pays a first record (measured ~11 us on the default line's critical path).
static constexpr size_t EVPOOL_WARM = 1024;
extern "C" int pvt_set_profiling_kernel(pvt_ctx* ctx, const char* kernel) {
  if (!ctx) return PVT_EINVAL;
  ctx->prof_only = kernel ? kernel : "";
  return PVT_OK;
}

extern "C" int pvt_set_profiling(pvt_ctx* ctx, int on) {
  if (!ctx) return PVT_EINVAL;
  ctx->profiling = on == 2 ? 2 : (on != 0 ? 1 : 0);
  if (ctx->profiling && ctx->evpool.size() + 2 * ctx->pending.size() < EVPOOL_WARM) {
    (void)hipSetDevice(ctx->device);
    while (ctx->evpool.size() + 2 * ctx->pending.size() < EVPOOL_WARM) {
      hipEvent_t e = nullptr;
      if (hipEventCreateWithFlags(&e, PROFILE_EVENT_FLAGS) != hipSuccess) break;
      (void)hipEventRecord(e, ctx->stream);
      ctx->evpool.push_back(e);
    }
    (void)hipStreamSynchronize(ctx->stream);
  }
  return PVT_OK;
}
extern "C" int pvt_reset_kstats(pvt_ctx* ctx) {
  if (!ctx) return PVT_EINVAL;
  (void)hipStreamSynchronize(ctx->stream);
  harvest(ctx);
  std::memset(ctx->ks, 0, sizeof(ctx->ks));
  ctx->kks.clear();
  return PVT_OK;
}
extern "C" int pvt_get_kstats(pvt_ctx* ctx, int kclass, pvt_kstats* out) {
  if (!ctx || !out || kclass < 0 || kclass >= PVT_K_COUNT) return PVT_EINVAL;
  (void)hipStreamSynchronize(ctx->stream);
  harvest(ctx);
  *out = ctx->ks[kclass];
  return PVT_OK;
}
extern "C" int pvt_get_kernel_kstats(pvt_ctx* ctx, const char* kernel, pvt_kstats* out) {
  if (!ctx || !kernel || !out) return PVT_EINVAL;
  (void)hipStreamSynchronize(ctx->stream);
  harvest(ctx);
  auto it = ctx->kks.find(kernel);
  if (it == ctx->kks.end()) std::memset(out, 0, sizeof(*out));
  else *out = it->second;
  return PVT_OK;
}
extern "C" int pvt_set_window(pvt_ctx* ctx, int tasks) {
  if (!ctx || tasks < 0) return PVT_EINVAL;
  ctx->window = std::min(tasks, MAX_WINDOW);
  return PVT_OK;
}
extern "C" int pvt_set_score_tw(pvt_ctx* ctx, int tw) {
  if (!ctx || (tw != 0 && tw != 2 && tw != 4)) return PVT_EINVAL;
  ctx->score_tw = tw;
  return PVT_OK;
}
extern "C" int pvt_set_pipeline(pvt_ctx* ctx, int on) {
  if (!ctx) return PVT_EINVAL;
  ctx->pipeline = on != 0;
  return PVT_OK;
}
extern "C" int pvt_set_epochs(pvt_ctx* ctx, int on) {
  if (!ctx) return PVT_EINVAL;
  ctx->epochs = on != 0;
  return PVT_OK;
}
extern "C" int pvt_epoch_stats(pvt_ctx* ctx, int64_t* epochs, int64_t* segments, int64_t* rejected) {
  if (!ctx) return PVT_EINVAL;
  if (epochs) *epochs = ctx->n_epochs;
  if (segments) *segments = ctx->n_segs;
  if (rejected) *rejected = ctx->n_rejected;
  return PVT_OK;
}
extern "C" int pvt_set_band(pvt_ctx* ctx, int32_t min_hosts) {
  if (!ctx || min_hosts < 0) return PVT_EINVAL;
  ctx->band_min = min_hosts;
  return PVT_OK;
}
extern "C" int pvt_set_zero_walk(pvt_ctx* ctx, int on) {
  if (!ctx) return PVT_EINVAL;
  ctx->zwalk = on != 0;
  return PVT_OK;
}
extern "C" int pvt_zero_walk_stats(pvt_ctx* ctx, int64_t* frontier_chains, int64_t* list_chains,
                                   int64_t* longest_chain) {
  if (!ctx) return PVT_EINVAL;
  if (frontier_chains) *frontier_chains = ctx->n_zchains;
  if (list_chains) *list_chains = ctx->n_gchains;
  if (longest_chain) *longest_chain = ctx->n_longest;
  return PVT_OK;
}
extern "C" int pvt_last_stats(pvt_ctx* ctx, int64_t* windows, int64_t* refills) {
  if (!ctx) return PVT_EINVAL;
  if (windows) *windows = ctx->windows;
  if (refills) *refills = ctx->refills;
  return PVT_OK;
}
// Diagnostic (not part of the public ABI): commit-walk phase cycle sums of a PVT_STAMPS build.
extern "C" int pvt_debug_commit_stamps(pvt_ctx* ctx, uint64_t* out, int n) {
  if (!ctx || !out || n < 8) return PVT_EINVAL;
#ifdef PVT_STAMPS
  // 32 counters, then per-round cycles of the resident kernel (4096 rounds)
  constexpr int NW = 32 + 4096;
  if (!ctx->stamps) {
    if (hipMalloc((void**)&ctx->stamps, sizeof(uint64_t) * NW) != hipSuccess) return PVT_ENOMEM;
    (void)hipMemset(ctx->stamps, 0, sizeof(uint64_t) * NW);
    std::memset(out, 0, sizeof(uint64_t) * std::min(n, NW));
    return PVT_OK;
  }
  if (hipMemcpy(out, ctx->stamps, sizeof(uint64_t) * std::min(n, NW), hipMemcpyDeviceToHost) != hipSuccess)
    return PVT_EHIP;
  return PVT_OK;
#else
  return PVT_EUNSUPPORTED;
#endif
}

// Diagnostic (not part of the public ABI): score-pass candidate counters of a PVT_DIAG build.
extern "C" int pvt_debug_score_counts(pvt_ctx* ctx, uint64_t* out, int n, int reset) {
  if (!ctx || !out || n < 5) return PVT_EINVAL;
  (void)hipSetDevice(ctx->device);
  return pvt::score_diag(out, n, reset);
}

extern "C" const char* pvt_last_error(pvt_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

// ---------------------------------------------------------------- round driver
// Host segments per task for the score pass: enough waves to fill 256 CUs (~16 per CU) when
// the window is short, at least 4096 hosts per segment, a multiple of 8 (one XCD per
// blockIdx % 8), capped by the segment-list scratch.
static constexpr size_t SEG_ENTRIES_MAX = (size_t)MAX_WINDOW * MAX_SEG * KL;
// vbp best-fit scores are continuous, so a segment's list keeps improving while it streams:
// about KL * (1 + ln(H / (S * KL))) serial insertions per segment, S times per task. Fewer,
// longer segments halve those insertions at 16 (measured: 29.7 -> 26.2 ms of score per
// 1M x 10k round); cost_aware's zero-cost zone fills its lists at once and wants the waves.
static int choose_segments(int H, int nt, int mode, int force_tw, bool epoch, int force_S) {
  const int tw = score_tasks_per_wave(mode, H, force_tw);
  const int task_waves = (nt + tw - 1) / tw;
  int S = (4096 + task_waves - 1) / task_waves;
  if (mode == PVT_VBP_BF) S = std::min(S, 16);
  // cost_aware best-fit over many tasks (epochs): each segment fills its list from the zero-cost
  // zones' lowest-index hosts and exits early, so fewer, longer segments stream fewer hosts per
  // task -- but a merged list of S x 64 entries must stay deep enough for a whole group's walk
  // (config 5 ca_bf epoch of 10k tasks: S = 2 -> 5.6 ms, 4 -> 4.1, 8 -> 4.8; S = 2 refills;
  // config 3, 1k tasks: 8 -> 0.82 ms, 4 -> 0.73)
  if (mode == PVT_CA_BF && epoch) S = 4;
  if (force_S > 0) S = force_S;   // (PVT_SEGMENTS, read at context creation)
  S = std::min(S, std::max(1, H / 4096));
  S = std::min(S, std::max(MAX_SEG, (int)(SEG_ENTRIES_MAX / ((size_t)nt * KL))));
  S = std::max(1, std::min(S, 256));
  if (S >= 8) S = S / 8 * 8;
  return S;
}
// keyed first-fit scan depth: entries per task list (deeper lists, fewer refills)
static constexpr int KSCAN_DEPTH = 256;
// zero-key prefix used alone (no sort) when it holds at least this many hosts
static constexpr int KPREFIX_MIN = 1024;
static double bytes_per_candidate(int mode) {
  // cost_aware 36 B (4 x fp64 avail + int32 zone); vbp best-fit 36 B
  // (+ host-id rank); opportunistic / vbp first-fit 32 B.
  return (mode == PVT_CA_FF || mode == PVT_CA_BF || mode == PVT_VBP_BF) ? 36.0 : 32.0;
}

// a2: processing order. Group-major (stable by group id), within a group caller order or, with
// sort_tasks, stable descending ||d||2. Two LSD passes of a stable radix sort.
// Processing order (a2). Grouped rounds take the optimistic path: group counts, offsets and the
// pinned copies of counts / anchors / cost table, then the per-group sorts, all launched with no
// synchronisation (*pending = true); the caller syncs once, later, and calls build_order_check.
// Spin on the count kernel's flag (the staged counts are visible once it holds flag_seq). Every
// 4096 polls the stream is queried: an idle stream with no flag is an error, never a hang.
static int wait_host_flag(pvt_ctx* ctx, volatile int32_t* f, int32_t seq, const char* what) {
  for (uint32_t n = 1;; n++) {
    if (__atomic_load_n(f, __ATOMIC_ACQUIRE) == seq) return PVT_OK;
    __builtin_ia32_pause();                   // (yield the core's pipeline to its sibling thread)
    if (n >= (1u << 18)) {
      // a long wait (the GPU is shared or the round is large): stop spinning and block on the
      // stream -- everything queued behind the kernel runs without the host
      HIPCHK(hipStreamSynchronize(ctx->stream));
      if (__atomic_load_n(f, __ATOMIC_ACQUIRE) == seq) return PVT_OK;
      return fail(ctx, PVT_EHIP, "%s: kernel finished without its flag", what);
    }
    if ((n & 4095) == 0) {
      const hipError_t e = hipStreamQuery(ctx->stream);
      if (e == hipSuccess) {
        if (__atomic_load_n(f, __ATOMIC_ACQUIRE) == seq) return PVT_OK;
        return fail(ctx, PVT_EHIP, "%s: kernel finished without its flag", what);
      }
      if (e != hipErrorNotReady) return fail(ctx, PVT_EHIP, "%s: %s", what, hipGetErrorString(e));
    }
  }
}
static int wait_stage_flag(pvt_ctx* ctx) {
  return wait_host_flag(ctx, ctx->flag_host, ctx->flag_seq, "grouped order");
}

static int build_order_radix(pvt_ctx* ctx, const pvt_round* r, int32_t** ord_out);
// hmin (or NULL): the frontier walk's host minima, written by the order's launch when it can
// (*hmin_done); stage_flag: the host then waits on ctx->flag_host instead of ev_stage.
static int build_order(pvt_ctx* ctx, const pvt_round* r, int32_t** ord_out, bool* pending,
                       double* hmin = nullptr, bool* hmin_done = nullptr,
                       ZoneWindows* zwin = nullptr) {
  *pending = false;
  if (hmin_done) *hmin_done = false;
  ctx->rs.stage_flag = false;
  const int T = r->n_tasks;
  hipStream_t st = ctx->stream;
  ENSURE(ctx->ord, sizeof(int32_t) * T);
  ENSURE(ctx->ord2, sizeof(int32_t) * T);
  int32_t* cur = P<int32_t>(ctx->ord);
  const bool grouped = r->task_group != nullptr && r->n_groups > 1;
  RoundState& R = ctx->rs;
  R.ginfo = false;
  R.zpre = false;
  if (grouped && r->n_groups <= (1 << 20)) {
    // one synchronisation: group counts, group anchors and the cost table to the host
    const int G = r->n_groups;
    const bool fused = T <= PREP_T_MAX && G <= GAGG_MAX;   // (launch_order_prep: two launches)
    if (!fused) {
      ENSURE(ctx->gcnt, sizeof(int32_t) * (G + 1));
      HIPCHK(hipMemsetAsync(ctx->gcnt.p, 0, sizeof(int32_t) * (G + 1), st));
      launch_group_hist(r->task_group, T, G, P<int32_t>(ctx->gcnt), st);
    }
    // staged in pinned memory: pageable destinations made each copy a ~20 us synchronous
    // staging step (profiles/r02q kernel trace)
    const bool ca = r->mode == PVT_CA_FF || r->mode == PVT_CA_BF;
    const size_t nz2 = ca ? (size_t)r->n_zones * r->n_zones : 0;
    const size_t need = sizeof(double) * nz2 + sizeof(int32_t) * (2 * (size_t)G + 1);
    if (ctx->gstage_cap < need) {
      if (ctx->gstage) (void)hipHostFree(ctx->gstage);
      ctx->gstage = nullptr;
      ctx->gstage_cap = 0;
      HIPCHK(hipHostMalloc(&ctx->gstage, need));
      ctx->gstage_cap = need;
    }
    // counts, anchors and cost table written into the pinned buffer by one kernel, which also
    // leaves the groups' offsets and scatter cursors on the device
    ENSURE(ctx->goff, sizeof(int32_t) * 2 * (G + 1));
    void* dstage = nullptr;
    HIPCHK(hipHostGetDevicePointer(&dstage, ctx->gstage, 0));
    double* dcst = reinterpret_cast<double*>(dstage);
    int32_t* dcnt = reinterpret_cast<int32_t*>(dcst + nz2);
    // the per-group sorts, optimistically (a group over GSORT_MAX tasks is left unsorted by the
    // kernel; build_order_check then redoes the order with radix passes)
    ENSURE(ctx->gskey, sizeof(uint64_t) * T);
    ENSURE(ctx->gsidx, sizeof(int32_t) * T);
    if (fused) {
      // placement fill and (cost_aware) zone tables too: round_begin skips its own
      if (ca) {
        ENSURE(ctx->csum, sizeof(double) * r->n_zones * r->n_zones);
        ENSURE(ctx->bsum, sizeof(double) * r->n_zones * r->n_zones);
      }
      PrepArgs pa{r->task_group, T, G, r->group_anchor, r->cost, r->bw, r->n_zones, (int)nz2,
                  r->dem, r->sort_tasks ? 1 : 0, r->placement, P<int32_t>(ctx->goff), dcnt,
                  dcnt + G + 1, dcst, ca ? P<double>(ctx->csum) : nullptr,
                  ca ? P<double>(ctx->bsum) : nullptr, P<uint64_t>(ctx->gskey), P<int32_t>(ctx->gsidx),
                  nullptr, 0};
      R.prep_fused = true;
      if (G <= GCOMPACT_MAX) {   // one launch: the counts (block 0) beside the sorted, gathered order
        // the host polls a flag the count block stores (no event: a marker on the stream cost
        // ~5 us of idle GPU between launches)
        pa.hflag = ctx->flag_hdev;
        pa.seq = ++ctx->flag_seq;
        R.stage_flag = true;
        const bool zw = hmin && zwin && ca && r->n_zones <= ZMAX;
        launch_group_sort_gather(pa, GatherOut{cur, P<double>(ctx->dem_ord), P<int32_t>(ctx->anc_ord),
                                               P<int32_t>(ctx->grp_ord), r->order, r->avail,
                                               r->n_hosts, hmin, ctx->stamps, r->zone,
                                               zw ? zwin : nullptr}, st);
        if (hmin_done) *hmin_done = hmin != nullptr;
        R.zpre = zw;
        R.gathered = true;
        R.ginfo = ca;
        *pending = true;
        *ord_out = cur;
        return PVT_OK;
      }
      launch_order_prep(pa, st, ctx->ev_stage);
    } else {
      launch_group_stage(P<int32_t>(ctx->gcnt), G, r->group_anchor, r->cost, (int)nz2,
                         P<int32_t>(ctx->goff), dcnt, dcnt + G + 1, dcst, st);
      HIPCHK(hipGetLastError());
      const uint64_t* keys = nullptr;
      if (r->sort_tasks) {
        ENSURE(ctx->keys64a, sizeof(uint64_t) * T);
        launch_norm_keys(r->dem, T, nullptr, P<uint64_t>(ctx->keys64a), st);
        keys = P<uint64_t>(ctx->keys64a);
      }
      launch_group_scatter(r->task_group, keys, T, G, P<int32_t>(ctx->goff) + G + 1,
                           P<uint64_t>(ctx->gskey), P<int32_t>(ctx->gsidx), st);
      HIPCHK(hipEventRecord(ctx->ev_stage, st));
    }
    // the host waits for the staged counts only (ev_stage), not for the scatter, sorts and
    // gathers queued after them: it plans the round while they run
    launch_group_sort(P<int32_t>(ctx->goff), G, P<uint64_t>(ctx->gskey), P<int32_t>(ctx->gsidx),
                      cur, st);
    R.ginfo = ca;
    *pending = true;
    *ord_out = cur;
    return PVT_OK;
  }
  return build_order_radix(ctx, r, ord_out);
}

// After the caller's synchronisation: the group counts, anchors and cost table the optimistic
// path staged; *redo = a group exceeded the LDS sort (the order must be rebuilt by radix passes).
static int build_order_check(pvt_ctx* ctx, const pvt_round* r, bool* redo) {
  RoundState& R = ctx->rs;
  const int G = r->n_groups;
  const bool ca = r->mode == PVT_CA_FF || r->mode == PVT_CA_BF;
  const size_t nz2 = ca ? (size_t)r->n_zones * r->n_zones : 0;
  const double* cst = reinterpret_cast<const double*>(ctx->gstage);
  const int32_t* cnt = reinterpret_cast<const int32_t*>(cst + nz2);
  const int32_t* gan = cnt + G + 1;
  R.gcnt.assign(cnt, cnt + G + 1);
  R.ga_host.assign(gan, gan + G);
  R.cost_host.assign(cst, cst + nz2);
  if (R.gcnt[G] != 0) return fail(ctx, PVT_EINVAL, "task_group out of range");
  int mx = 0;
  for (int g = 0; g < G; g++) mx = std::max(mx, R.gcnt[g]);
  *redo = mx > GSORT_MAX;
  return PVT_OK;
}

// Processing order by radix passes: stable by descending norm (sort_tasks), then stable by group.
static int build_order_radix(pvt_ctx* ctx, const pvt_round* r, int32_t** ord_out) {
  const int T = r->n_tasks;
  hipStream_t st = ctx->stream;
  int32_t* cur = P<int32_t>(ctx->ord);
  int32_t* alt = P<int32_t>(ctx->ord2);
  const bool grouped = r->task_group != nullptr && r->n_groups > 1;
  launch_iota(cur, T, st);
  if (r->sort_tasks) {
    ENSURE(ctx->keys64a, sizeof(uint64_t) * T);
    ENSURE(ctx->keys64b, sizeof(uint64_t) * T);
    launch_norm_keys(r->dem, T, nullptr, P<uint64_t>(ctx->keys64a), st);
    size_t tmp = 0;
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, P<uint64_t>(ctx->keys64a),
                                              P<uint64_t>(ctx->keys64b), cur, alt, T, 0, 64, st));
    ENSURE(ctx->sorttmp, tmp);
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(ctx->sorttmp.p, tmp, P<uint64_t>(ctx->keys64a),
                                              P<uint64_t>(ctx->keys64b), cur, alt, T, 0, 64, st));
    std::swap(cur, alt);
  }
  if (grouped) {
    ENSURE(ctx->keys32a, sizeof(uint32_t) * T);
    ENSURE(ctx->keys32b, sizeof(uint32_t) * T);
    launch_group_keys(r->task_group, cur, T, P<uint32_t>(ctx->keys32a), st);
    int bits = 1;
    while ((1 << bits) < r->n_groups && bits < 31) bits++;
    size_t tmp = 0;
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, P<uint32_t>(ctx->keys32a),
                                              P<uint32_t>(ctx->keys32b), cur, alt, T, 0, bits, st));
    ENSURE(ctx->sorttmp, tmp);
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(ctx->sorttmp.p, tmp, P<uint32_t>(ctx->keys32a),
                                              P<uint32_t>(ctx->keys32b), cur, alt, T, 0, bits, st));
    std::swap(cur, alt);
  }
  *ord_out = cur;
  return PVT_OK;
}

static int check_round(pvt_ctx* ctx, const pvt_round* r) {
  if (!r) return fail(ctx, PVT_EINVAL, "null round");
  if (r->reserved != 0) return fail(ctx, PVT_EINVAL, "reserved must be 0");
  if (r->n_hosts < 1 || r->n_tasks < 0 || r->n_zones < 1 || r->n_zones > ZMAX)
    return fail(ctx, PVT_EINVAL, "bad sizes H=%d T=%d Z=%d", r->n_hosts, r->n_tasks, r->n_zones);
  if (r->mode < PVT_CA_FF || r->mode > PVT_VBP_BF) return fail(ctx, PVT_EINVAL, "bad mode %d", r->mode);
  if (!r->avail || !r->zone) return fail(ctx, PVT_EINVAL, "null host array");
  if (r->n_tasks > 0 && (!r->dem || !r->order || !r->placement))
    return fail(ctx, PVT_EINVAL, "null task array");
  if ((r->mode == PVT_CA_FF || r->mode == PVT_CA_BF) && (!r->cost || !r->bw))
    return fail(ctx, PVT_EINVAL, "cost_aware needs cost and bw");
  if (r->n_tasks > 0 && r->task_group && (r->n_groups < 1 || !r->group_anchor))
    return fail(ctx, PVT_EINVAL, "task_group needs n_groups >= 1 and group_anchor");
  if (r->mode == PVT_VBP_BF && !r->tiebreak) return fail(ctx, PVT_EINVAL, "vbp best-fit needs tiebreak");
  if (r->mode == PVT_OPP && !r->mt_state) return fail(ctx, PVT_EINVAL, "opportunistic needs mt_state");
  if (r->mode == PVT_CA_BF && r->decay && r->n_tasks > 0)
    return fail(ctx, PVT_EUNSUPPORTED, "cost_aware best-fit with host_decay (reference crashes, cost_aware.py:26,81)");
  return PVT_OK;
}

static void lists_from(pvt_ctx* ctx, Lists& L, int b = 0) {
  L.e = P<ListEntry>(ctx->l_e[b]);
  L.ids = P<int32_t>(ctx->l_ids[b]);
  L.t = P<TaskRec>(ctx->l_t[b]);
}

// Opportunistic: windows of OPP_MAXW tasks in caller order; count pass then commit walk. The
// MT19937 state travels host -> device -> host around the round.
static int opp_round(pvt_ctx* ctx, const pvt_round* r) {
  const int T = r->n_tasks, H = r->n_hosts;
  hipStream_t st = ctx->stream;
  // Window: longer windows cut the per-window launches and hand-offs; the walk's touched-host
  // tables bound them (OPP_MAXW, LDS). (bench sweeps at 1M hosts x 10k tasks: round 2 with the
  // speculative-range walk, profiles/r02h: pipelined 64 -> 20.1 ms, 128 -> 18.5, 256 -> 19.4;
  // round 4 with the register-row walk: 128 -> 10.0, 256 -> 9.6)
  const int wdef = ctx->pipeline ? OPP_WINDOW_PIPE : OPP_WINDOW_DEFAULT;
  const int W = std::max(1, std::min(ctx->window > 0 ? ctx->window : wdef, OPP_MAXW));
  const int nq = (H + OPP_CH - 1) / OPP_CH, nsq = (nq + OPP_SUP - 1) / OPP_SUP;
  ENSURE(ctx->dem_ord, sizeof(double) * 4 * T);
  ENSURE(ctx->anc_ord, sizeof(int32_t) * T);
  launch_gather_tasks(r->dem, r->order, nullptr, nullptr, T, P<double>(ctx->dem_ord),
                      P<int32_t>(ctx->anc_ord), nullptr, st);
  // Pipelined windows (a walk's inherited + own touched hosts, 2 x OPP_MAXW, fit its LDS):
  // window k+1's count pass runs on the side stream while window k is walked. Walk k leaves
  // global availability untouched and hands its hosts to walk k+1, which applies them on entry
  // and then releases count k+2; so every count pass reads the capacities its walk's
  // predecessor started from, and the hosts that walk touched are touched for the next walk.
  const int nwin = (T + W - 1) / W;
  const bool pipe = ctx->pipeline && nwin > 1;
  const int nbuf = pipe ? 2 : 1;
  const size_t bm_bytes = sizeof(uint64_t) * 4 * (size_t)nq * W;
  const size_t sc_bytes = sizeof(int32_t) * (size_t)nsq * W;
  const size_t tl_bytes = pipe ? sizeof(OppTouched) : 0;
  const size_t slot = (bm_bytes + sc_bytes + tl_bytes + 255) / 256 * 256;
  ENSURE(ctx->opp, slot * nbuf + sizeof(uint32_t) * 640);
  ENSURE(ctx->oppfault, 16);
  int32_t* fault = P<int32_t>(ctx->oppfault);
  HIPCHK(hipMemsetAsync(fault, 0, sizeof(int32_t), st));
  char* base = reinterpret_cast<char*>(ctx->opp.p);
  auto bm_of = [&](int b) { return reinterpret_cast<uint64_t*>(base + slot * b); };
  auto sc_of = [&](int b) { return reinterpret_cast<int32_t*>(base + slot * b + bm_bytes); };
  auto tl_of = [&](int b) { return reinterpret_cast<OppTouched*>(base + slot * b + bm_bytes + sc_bytes); };
  uint32_t* mt = reinterpret_cast<uint32_t*>(base + slot * nbuf);
  HIPCHK(hipMemcpyAsync(mt, r->mt_state, sizeof(uint32_t) * 625, hipMemcpyHostToDevice, st));
  const double bpc = bytes_per_candidate(r->mode);
  auto count = [&](int k, hipStream_t s) {
    const int t0 = k * W, nt = std::min(W, T - t0);
    OppCountArgs ca{r->avail, P<double>(ctx->dem_ord) + (size_t)t0 * 4, H, nt, 0, 0, nq, nsq,
                    W, bm_of(k % nbuf), sc_of(k % nbuf), 0, nsq, nq, nsq};
    Scope sc(ctx, PVT_K_SCORE, (double)nt * H, (double)nt * H * bpc, s, "opp_count_kernel");
    launch_opp_count(ca, s);
  };
  if (nwin > 0) count(0, st);
  for (int k = 0; k < nwin; k++) {
    const int t0 = k * W, nt = std::min(W, T - t0);
    const bool next = pipe && k + 1 < nwin;
    ctx->windows++;
    if (!pipe && k > 0) count(k, st);   // sequential: window k counted after walk k-1 wrote back
    const OppTouched* in = (pipe && k > 0) ? tl_of((k - 1) % nbuf) : nullptr;
    if (in) launch_opp_apply(in, r->avail, H, st);   // walk k-1's commits, before count k+1
    if (next) {
      HIPCHK(hipEventRecord(ctx->ev_walk, st));
      HIPCHK(hipStreamWaitEvent(ctx->side, ctx->ev_walk, 0));
      count(k + 1, ctx->side);
      HIPCHK(hipEventRecord(ctx->ev_lists, ctx->side));
    }
    OppCommitArgs oa{r->avail, P<double>(ctx->dem_ord) + (size_t)t0 * 4, bm_of(k % nbuf),
                     sc_of(k % nbuf), H, nt, nq, nsq, W, r->placement + t0, mt, ctx->stamps,
                     in, next ? tl_of(k % nbuf) : nullptr, next ? 0 : 1, fault};
    {
      Scope s(ctx, PVT_K_COMMIT, 0, 0, nullptr, "opp_commit_kernel");
      launch_opp_commit(oa, st);
    }
    if (next) HIPCHK(hipStreamWaitEvent(st, ctx->ev_lists, 0));
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(r->mt_state, mt, sizeof(uint32_t) * 625, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(ctx->next_host + 3, fault, sizeof(int32_t), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (ctx->next_host[3])
    return fail(ctx, PVT_EHIP, "opportunistic walk: inconsistent feasible counts (a range's first "
                "task, window-local %d, failed its verification)", ctx->next_host[3] - 1);
  return PVT_OK;
}

// vbp best-fit band lists: hosts [lo, hi) sorted by snapshot memory (stable radix sort of the
// orderable bits of avail[1]) and their snapshot state gathered in that order; no host touched.
// (rocPRIM's onesweep sort measured slower than the default dispatch's merge sort at config 5's
// 1M hosts: 8 passes of ~25 us plus two fill launches each, against ~0.19 ms; the memory values
// of uniform random hosts vary in ~63 key bits, so no pass can be skipped.)
static int band_snapshot(pvt_ctx* ctx) {
  RoundState& R = ctx->rs;
  const pvt_round* r = &R.r;
  hipStream_t st = ctx->stream;
  const int n = R.hi - R.lo;
  ENSURE(ctx->bkey, sizeof(uint64_t) * 2 * (size_t)n);
  ENSURE(ctx->bidx, sizeof(int32_t) * 2 * (size_t)n);
  ENSURE(ctx->bsa, sizeof(double) * 4 * (size_t)n);
  ENSURE(ctx->bstb, sizeof(uint32_t) * (size_t)n);
  ENSURE(ctx->btouch, (size_t)R.H);
  ENSURE(ctx->btlist, sizeof(int32_t) * (size_t)R.H);
  ENSURE(ctx->btcnt, 16);
  ENSURE(ctx->bpos, sizeof(int32_t) * (size_t)R.H);
  ENSURE(ctx->bptouch, (size_t)n);
  ENSURE(ctx->brec, sizeof(BandRec) * (size_t)n);
  uint64_t* k0 = P<uint64_t>(ctx->bkey);
  int32_t* i0 = P<int32_t>(ctx->bidx);
  size_t tmp = 0;
  HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, k0, k0 + n, i0, i0 + n, n, 0, 64, st));
  ENSURE(ctx->bsorttmp, tmp);
  const int bs = ctx->t_band_segs ? ctx->t_band_segs : BAND_SEGS;   // (PVT_BAND_SEGS: 2 ... 32)
  R.band_S = (bs == 1 || bs == 2 || bs == 4 || bs == 8 || bs == 16 || bs == 32) ? bs : BAND_SEGS;
  Scope sc(ctx, PVT_K_OTHER, 0, 0);
  launch_band_keys(r->avail, r->tiebreak, R.H, R.lo, n, k0, i0, P<BandRec>(ctx->brec), st);
  HIPCHK(hipcub::DeviceRadixSort::SortPairs(ctx->bsorttmp.p, tmp, k0, k0 + n, i0, i0 + n, n, 0, 64, st));
  launch_band_gather(P<BandRec>(ctx->brec), R.lo, n, i0 + n, P<double>(ctx->bsa),
                     P<uint32_t>(ctx->bstb), P<int32_t>(ctx->bpos), st);
  HIPCHK(hipMemsetAsync(ctx->btouch.p, 0, (size_t)R.H, st));
  HIPCHK(hipMemsetAsync(ctx->bptouch.p, 0, (size_t)n, st));
  HIPCHK(hipMemsetAsync(ctx->btcnt.p, 0, 16, st));
  HIPCHK(hipGetLastError());
  return PVT_OK;
}

// The last walk's committed hosts flagged and listed as touched (band lists), on the context's
// stream. Called only where no band score pass is in flight (it would read the touched table).
static void flush_touched(pvt_ctx* ctx) {
  RoundState& R = ctx->rs;
  if (!R.band || R.touch_lb < 0) return;
  launch_touch_update(P<int32_t>(ctx->owned[R.touch_lb]),
                      R.touch_status ? R.touch_status : P<int32_t>(ctx->next),
                      P<uint8_t>(ctx->btouch), P<int32_t>(ctx->btlist), P<int32_t>(ctx->btcnt),
                      P<int32_t>(ctx->bpos), R.lo, R.hi, P<uint8_t>(ctx->bptouch), ctx->stream);
  R.touch_lb = -1;
}

// ---------------------------------------------------------------- round state machine
// pvt_place() and the sharded calls share one round: begin (order, gathers, zone tables, group
// boundaries), then per window: candidate lists over this context's host range (optionally
// exchanged between ranks), then the commit walk, which decides where the next window starts.
static int zero_cost_components(pvt_ctx* ctx);

static int round_begin(pvt_ctx* ctx, const pvt_round* rin, int lo, int hi, int world) {
  RoundState& R = ctx->rs;
  R.active = false;
  int rc = check_round(ctx, rin);
  if (rc) return rc;
  R.r = *rin;
  const pvt_round* r = &R.r;
  ctx->windows = ctx->refills = 0;
  HIPCHK(hipSetDevice(ctx->device));
  const int T = r->n_tasks, H = r->n_hosts, Z = r->n_zones;
  R.T = T; R.H = H; R.Z = Z; R.lo = lo; R.hi = hi; R.world = world;
  R.t0 = 0; R.g = 0; R.nt = 0; R.lb = 0;
  R.gstart.assign(1, 0);
  R.ganchor.clear();
  R.gid.clear();
  if (T == 0) { R.ngroups = 0; R.active = true; return PVT_OK; }
  hipStream_t st = ctx->stream;

  bool pending = false;
  R.prep_fused = false;
  R.gathered = false;
  ENSURE(ctx->dem_ord, sizeof(double) * 4 * T);
  ENSURE(ctx->anc_ord, sizeof(int32_t) * T);
  ENSURE(ctx->grp_ord, sizeof(int32_t) * T);
  // a cost_aware best-fit round of epochs (epoch_groups) starts with the frontier walk's host
  // minima: written by the grouped order's launch, or queued below, they are ready while the
  // host waits for the grouped order's counts
  const bool want_hmin = ctx->epochs && ctx->zwalk && r->mode == PVT_CA_BF && r->task_group &&
                         r->n_groups >= 2 && T >= 2 && !r->rt_bw && Z <= ZMAX && world == 1;
  if (want_hmin) {
    ENSURE(ctx->hmin, sizeof(double) * 4 * ZW_MIN_PARTS);
    if (ctx->t_zpre) ENSURE(ctx->zwin, sizeof(ZoneWindows));
  }
  bool hmin_done = false;
  if ((rc = build_order(ctx, r, &R.ord, &pending, want_hmin ? P<double>(ctx->hmin) : nullptr,
                        &hmin_done, want_hmin && ctx->t_zpre ? P<ZoneWindows>(ctx->zwin) : nullptr)))
    return rc;
  if (!R.prep_fused) HIPCHK(hipMemsetAsync(r->placement, 0xff, sizeof(int32_t) * T, st));
  auto order_out = [&]() -> int {   // (the gather also writes the caller's order)
    launch_gather_tasks(r->dem, R.ord, r->task_group, r->group_anchor, T, P<double>(ctx->dem_ord),
                        P<int32_t>(ctx->anc_ord), P<int32_t>(ctx->grp_ord), st, r->n_groups, r->order);
    return PVT_OK;
  };
  if (!R.gathered && (rc = order_out())) return rc;
  const bool ca = r->mode == PVT_CA_FF || r->mode == PVT_CA_BF;
  if (ca) {
    ENSURE(ctx->csum, sizeof(double) * Z * Z);
    ENSURE(ctx->bsum, sizeof(double) * Z * Z);
    if (!R.prep_fused)
      launch_zone_tables(r->cost, r->bw, Z, P<double>(ctx->csum), P<double>(ctx->bsum), st);
  }
  R.hmin_pre = false;
  if (want_hmin) {
    if (!hmin_done) {
      Scope sc(ctx, PVT_K_OTHER, 0, 0);
      launch_host_min(r->avail, H, 0, H, P<double>(ctx->hmin), st);
    }
    R.hmin_pre = true;
  }
  if (pending) {   // the one synchronisation of the grouped order: counts, anchors, cost table
    if (R.stage_flag) {
      if ((rc = wait_stage_flag(ctx))) return rc;
    } else {
      HIPCHK(hipEventSynchronize(ctx->ev_stage));
    }
    bool redo = false;
    if ((rc = build_order_check(ctx, r, &redo))) return rc;
    if (redo) {
      if ((rc = build_order_radix(ctx, r, &R.ord))) return rc;
      if ((rc = order_out())) return rc;
    }
  }

  // group boundaries in processing order (only cost_aware first-fit with sort_hosts needs them)
  R.keyed = r->mode == PVT_CA_FF && r->sort_hosts;
  R.kscan = false;
  R.kmode = 0; R.kn = 0; R.kstall = false;
  R.ordered = (r->mode == PVT_VBP_FF) || (r->mode == PVT_CA_FF && !r->sort_hosts);
  if (R.keyed) {
    std::vector<int32_t> tg, ga;
    if (r->task_group) {
      std::vector<int> cnt(r->n_groups, 0);
      if (R.ginfo) {                          // copied by build_order
        for (int g = 0; g < r->n_groups; g++) cnt[g] = R.gcnt[g];
        ga = R.ga_host;
      } else {
        tg.resize(T);
        ga.resize(r->n_groups);
        HIPCHK(hipMemcpyAsync(tg.data(), r->task_group, sizeof(int32_t) * T, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(ga.data(), r->group_anchor, sizeof(int32_t) * r->n_groups,
                              hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        for (int t = 0; t < T; t++) {
          if (tg[t] < 0 || tg[t] >= r->n_groups) return fail(ctx, PVT_EINVAL, "task_group out of range");
          cnt[tg[t]]++;
        }
      }
      int off = 0;
      R.gstart.clear();
      for (int g = 0; g < r->n_groups; g++) {
        if (cnt[g] == 0) continue;
        R.gstart.push_back(off);
        R.ganchor.push_back(ga[g]);
        R.gid.push_back(g);
        off += cnt[g];
      }
    } else {
      R.ganchor.push_back(0);
      R.gid.push_back(0);
    }
    ENSURE(ctx->key, sizeof(double) * H);
    ENSURE(ctx->next, sizeof(int32_t) * 4);
    R.kscan = ctx->keyed_scan != 0;
    if (ctx->t_keyed_scan >= 0) R.kscan = ctx->t_keyed_scan != 0;   // (PVT_KEYED_SCAN)
    if (R.kscan && hi > lo) {
      const int n = hi - lo;
      ENSURE(ctx->kskey, sizeof(uint64_t) * 2 * (size_t)std::max(n, 1));
      ENSURE(ctx->kperm, sizeof(int32_t) * (size_t)std::max(n, 1));
      ENSURE(ctx->kiota, sizeof(int32_t) * (size_t)std::max(n, 1));
      size_t tmp = 0;
      HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, P<uint64_t>(ctx->kskey),
                                                P<uint64_t>(ctx->kskey) + n, P<int32_t>(ctx->kiota),
                                                P<int32_t>(ctx->kperm), n, 0, 64, st));
      size_t tmp2 = 0;
      HIPCHK(hipcub::DeviceSelect::Flagged(nullptr, tmp2, P<int32_t>(ctx->kiota),
                                           P<uint8_t>(ctx->kflag), P<int32_t>(ctx->kperm),
                                           P<int32_t>(ctx->next) + 2, n, st));
      ENSURE(ctx->ksorttmp, std::max(tmp, tmp2));
      ENSURE(ctx->kflag, (size_t)n);
      launch_iota(P<int32_t>(ctx->kiota), n, st);
    }
  }
  // vbp first-fit / unsorted cost_aware first-fit: the frontier walk over the first alive hosts
  // (ordered_frontier); its scratch is the keyed path's (the modes exclude each other)
  R.sh_epochs = false;
  R.list_until = 0;
  R.ofront = ctx->zwalk && R.ordered && T >= ORDERED_FRONTIER_MIN && H >= 64;
  R.of_try = R.ofront;
  R.of_tasks = ctx->of_tasks;
  R.kf_pending = false;
  if (R.ofront) {
    R.ofh = ORDERED_FRONTIER_HOSTS;
    if (ctx->t_of_hosts) R.ofh = ctx->t_of_hosts;   // (PVT_OF_HOSTS)
    ENSURE(ctx->next, sizeof(int32_t) * 4);
    ENSURE(ctx->kperm, sizeof(int32_t) * (size_t)H);
    ENSURE(ctx->kiota, sizeof(int32_t) * (size_t)H);
    ENSURE(ctx->kflag, (size_t)H);
    ENSURE(ctx->hmin, sizeof(double) * 4 * ZW_MIN_PARTS);
    size_t tmp2 = 0;
    HIPCHK(hipcub::DeviceSelect::Flagged(nullptr, tmp2, P<int32_t>(ctx->kiota), P<uint8_t>(ctx->kflag),
                                         P<int32_t>(ctx->kperm), P<int32_t>(ctx->next) + 2, H, st));
    ENSURE(ctx->ksorttmp, tmp2);
    launch_iota(P<int32_t>(ctx->kiota), H, st);
  }
  R.gstart.push_back(T);
  R.ngroups = R.keyed ? R.ganchor.size() : 1;
  // keyed first-fit: zero-key epochs (ff_epoch) over the groups, unsharded rounds
  R.ffe = false;
  R.ffe_skip = -1;
  if (R.keyed && !R.sharded && ctx->zwalk && ctx->epochs && !r->rt_bw && Z <= ZMAX &&
      T >= KEYED_FRONTIER_MIN) {
    R.egs = R.gstart;
    R.ega = R.ganchor;
    if ((rc = zero_cost_components(ctx))) return rc;
    R.ffe = true;
  }
  R.key_group = -1;
  R.touch_lb = -1;
  R.band = r->mode == PVT_VBP_BF && ctx->band_min > 0 && hi - lo >= ctx->band_min;
  if (R.band && (rc = band_snapshot(ctx))) return rc;
  R.runs.clear();
  if (R.band && ctx->lwalk && !R.sharded) {
    // representative list rows: the round's runs of equal demands, once (their ids on the host
    // size each window's rows; one synchronisation per round instead of a launch per window)
    ENSURE(ctx->brun, sizeof(int32_t) * (size_t)T);
    ENSURE(ctx->brdem, sizeof(double) * 4 * (size_t)T);
    launch_band_runs(P<double>(ctx->dem_ord), T, P<int32_t>(ctx->brun), P<double>(ctx->brdem), st);
    HIPCHK(hipGetLastError());
    R.runs.resize(T);
    HIPCHK(hipMemcpyAsync(R.runs.data(), ctx->brun.p, sizeof(int32_t) * (size_t)T,
                          hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }

  // Windows adapt to how far commit walks get before a list is exhausted: a walk that stops
  // early means the next window only needs about that many tasks (the score pass costs the
  // same per task either way, so short windows waste less on tasks that get re-scored).
  // default window: MAX_WINDOW for every policy. (vbp best-fit had 512: its walks search deeper
  // lists as a window's touched hosts pile up at the top of every task's ranking; with the
  // merge-path merge the longer windows win -- config 5: 3.33 ms at 512, 3.26 at 768, 3.07 at
  // 1024, round 4 sweep.)
  const int wdef = MAX_WINDOW;
  R.Wmax = std::max(1, std::min(ctx->window > 0 ? ctx->window : wdef, MAX_WINDOW));
  R.W = R.Wmax;
  ENSURE(ctx->seg, sizeof(SegEntry) * (size_t)SEG_ENTRIES_MAX);
  ENSURE(ctx->seg_feas, sizeof(int32_t) * (size_t)SEG_ENTRIES_MAX / KL);
  for (int b = 0; b < 2; b++) {
    ENSURE(ctx->l_e[b], sizeof(ListEntry) * (size_t)R.Wmax * LMAX);
    ENSURE(ctx->l_ids[b], sizeof(int32_t) * (size_t)R.Wmax * LMAX);
    ENSURE(ctx->l_t[b], sizeof(TaskRec) * (size_t)R.Wmax);
    ENSURE(ctx->owned[b], sizeof(int32_t) * MAX_WINDOW);
  }
  ENSURE(ctx->next, sizeof(int32_t) * 4);
  R.active = true;
  return PVT_OK;
}

// End of the group holding task t0 (keyed first-fit: windows never cross a group).
static int group_end(const RoundState& R, int t0) {
  if (!R.keyed) return R.T;
  size_t g = 0;
  while (g < R.ngroups && t0 >= R.gstart[g + 1]) g++;
  return g < R.ngroups ? R.gstart[g + 1] : R.T;
}

// Full stable radix sort of the frozen keys of this context's hosts (cost_aware.py:118-119).
static int keyed_full_sort(pvt_ctx* ctx) {
  RoundState& R = ctx->rs;
  const int n = R.hi - R.lo;
  size_t tmp = ctx->ksorttmp.n;
  const uint64_t* kin = reinterpret_cast<const uint64_t*>(P<double>(ctx->key) + R.lo);
  HIPCHK(hipcub::DeviceRadixSort::SortPairs(P<void>(ctx->ksorttmp), tmp, kin,
                                            P<uint64_t>(ctx->kskey) + n, P<int32_t>(ctx->kiota),
                                            P<int32_t>(ctx->kperm), n, 0, 64, ctx->stream));
  R.kmode = 2;
  R.kn = n;
  return PVT_OK;
}

static int ff_epoch(pvt_ctx* ctx, int* adv_out);

// Size of the next window at R.t0 (0: the round is done). Computes the frozen first-fit key of
// this context's hosts at a group start (cost_aware.py:118-119, on the current capacities).
// Keyed rounds first try zero-key epochs at each group start (ff_epoch): whole groups proven by
// the first-fit chain walk need no key at all.
static int round_next_window(pvt_ctx* ctx, int* nt_out) {
  RoundState& R = ctx->rs;
  *nt_out = 0;
  if (!R.active) return fail(ctx, PVT_EINVAL, "no round in progress");
  for (;;) {                      // (a group the keyed frontier walk completed: the next one)
  while (R.g < R.ngroups && R.t0 >= (R.keyed ? R.gstart[R.g + 1] : R.T)) R.g++;
  if (R.g >= R.ngroups || R.T == 0) return PVT_OK;
  const int ge = R.keyed ? R.gstart[R.g + 1] : R.T;
  int rc = 0;
  if (R.ffe && R.t0 == R.gstart[R.g] && R.key_group != (int)R.g && R.ffe_skip != (int)R.g) {
    int adv = 0;
    if ((rc = ff_epoch(ctx, &adv))) return rc;
    if (adv > 0) { R.t0 += adv; continue; }
    R.ffe_skip = (int)R.g;          // (this group goes to the keyed path below)
  }
  if (R.kstall) {                 // same group, frozen keys: complete the order
    R.kstall = false;
    if (R.key_group == (int)R.g && R.kmode == 1 && (rc = keyed_full_sort(ctx))) return rc;
  }
  if (R.keyed && R.key_group != (int)R.g && R.hi == R.lo && R.kscan && R.sharded) {
    // a rank with no hosts: no key, an empty prefix -- but the group start's frontier walk is a
    // collective step every rank takes (round_next_window decides it the same way everywhere)
    R.kf_pending = ctx->zwalk && R.t0 == R.gstart[R.g] && ge - R.t0 >= KEYED_FRONTIER_MIN &&
                   !R.r.rt_bw && R.Z <= ZMAX;
    HIPCHK(hipMemsetAsync(P<int32_t>(ctx->next) + 2, 0, sizeof(int32_t), ctx->stream));
    R.key_group = (int)R.g;
  }
  if (R.keyed && R.key_group != (int)R.g && R.hi > R.lo) {
    KeyArgs ka{R.r.avail, R.r.zone, R.r.decay, P<double>(ctx->csum), P<double>(ctx->bsum), R.H, R.Z,
               R.ganchor[R.g], R.lo, R.hi, P<double>(ctx->key),
               R.r.rt_bw ? R.r.rt_bw + (size_t)R.gid[R.g] * R.H : nullptr};
    {
      Scope sc(ctx, PVT_K_OTHER, 0, 0);
      launch_key(ka, ctx->stream);
    }
    if (R.kscan) {
      // The group's host order (cost_aware.py:118-119). Hosts of zero key (the anchor zone's:
      // no egress cost) come first, in host order; when there are enough of them the rest is
      // sorted only if a walk ever exhausts that prefix (kstall).
      const int n = R.hi - R.lo;
      const double* kin = P<double>(ctx->key) + R.lo;
      {
        Scope sc(ctx, PVT_K_OTHER, 0, 0);
        launch_zero_key_flags(kin, n, P<uint8_t>(ctx->kflag), ctx->stream);
        size_t tmp = ctx->ksorttmp.n;
        HIPCHK(hipcub::DeviceSelect::Flagged(P<void>(ctx->ksorttmp), tmp, P<int32_t>(ctx->kiota),
                                             P<uint8_t>(ctx->kflag), P<int32_t>(ctx->kperm),
                                             P<int32_t>(ctx->next) + 2, n, ctx->stream));
      }
      // The frontier walk (pvt_zwalk.hip, keyed mode) takes the group's first tasks from the
      // group start: each takes the first prefix host, in host order, that strictly fits, which
      // is the keyed order's answer whatever the prefix length (zero-key hosts lead it in both
      // modes below); it stops at the first task no host of the prefix's first ZW_M fits, and
      // the windowed list path goes on from there with the same frozen key. Launched on the
      // prefix length as the device holds it, read back with it in one synchronisation.
      const int n_g = ge - R.t0;
      const bool zk_any = ctx->zwalk && R.t0 == R.gstart[R.g] && n_g >= KEYED_FRONTIER_MIN &&
                          !R.r.rt_bw && R.Z <= ZMAX;
      const bool zk = zk_any && !R.sharded;
      // host-sharded: the walk runs on the merged window of every rank's first prefix hosts
      // (pvt_shard_score packs this rank's, PK_KEYED), after the prefix lengths are known
      R.kf_pending = zk_any && R.sharded;
      if (zk) {
        ENSURE(ctx->wres, sizeof(WinRec) * (size_t)n_g);
        const pvt_round* r = &R.r;
        ZwalkArgs za{r->avail, r->zone, R.H, R.Z, P<double>(ctx->dem_ord) + (size_t)R.t0 * 4,
                     P<int32_t>(ctx->anc_ord) + R.t0, R.ord + R.t0, P<double>(ctx->csum),
                     P<double>(ctx->bsum), nullptr, nullptr, P<int32_t>(ctx->next),
                     P<WinRec>(ctx->wres), r->placement, nullptr, ctx->stamps,
                     P<int32_t>(ctx->kperm), 0, R.lo, n_g, r->avail, P<int32_t>(ctx->next) + 2};
        Scope sc(ctx, PVT_K_COMMIT, 0, 0, nullptr, "zwalk_kernel");
        launch_zwalk_keyed(za, true, ctx->stream);
      }
      HIPCHK(hipGetLastError());
      HIPCHK(hipMemcpyAsync(ctx->next_host, P<int32_t>(ctx->next), sizeof(int32_t) * 3,
                            hipMemcpyDeviceToHost, ctx->stream));
      HIPCHK(hipStreamSynchronize(ctx->stream));
      const int nz = ctx->next_host[2];
      if (zk) {
        const int done = ctx->next_host[0];
        if (done < 0 || done > n_g)
          return fail(ctx, PVT_EHIP, "keyed frontier walk returned %d of %d", done, n_g);
        ctx->n_zchains += done > 0;
        R.t0 += done;
      }
      if (nz >= KPREFIX_MIN && nz < n) {
        R.kmode = 1;
        R.kn = nz;
        HIPCHK(hipMemsetAsync(P<uint64_t>(ctx->kskey) + n, 0, sizeof(uint64_t) * nz, ctx->stream));
      } else {
        if ((rc = keyed_full_sort(ctx))) return rc;
      }
    }
    R.key_group = (int)R.g;
  }
  if (R.t0 >= ge) continue;       // the frontier walk took the whole group
  R.nt = std::min(R.W, ge - R.t0);
  *nt_out = R.nt;
  return PVT_OK;
  }
}

// Exact candidate lists of tasks [t0, t0 + nt) over hosts [lo, hi) into list buffer `lb`, on
// stream `st`.
static int window_lists(pvt_ctx* ctx, int t0, int nt, int lb, hipStream_t st,
                        const int32_t* gate = nullptr) {
  RoundState& R = ctx->rs;
  const pvt_round* r = &R.r;
  const int Hl = R.hi - R.lo;
  ctx->windows++;
  Lists L;
  lists_from(ctx, L, lb);
  const double bpc = bytes_per_candidate(r->mode);
  const double* dem_w = P<double>(ctx->dem_ord) + (size_t)t0 * 4;
  const int32_t* anc_w = P<int32_t>(ctx->anc_ord) + t0;
  if (R.kscan) {
    const int n = R.hi - R.lo;
    PermArgs pa{r->avail, r->zone, P<uint64_t>(ctx->kskey) + n, P<int32_t>(ctx->kperm), dem_w,
                anc_w, R.ord + t0, R.H, nt, n > 0 ? R.kn : 0, KSCAN_DEPTH, R.lo,
                R.kmode == 1 ? 1 : 0, std::numeric_limits<double>::denorm_min(), L};
    Scope sc(ctx, PVT_K_SCORE, (double)nt * Hl, (double)nt * Hl * bpc, st, "perm_scan_kernel");
    launch_perm_scan(pa, st);
  } else if (R.ordered) {
    OrderedArgs oa{r->avail, r->zone, dem_w, anc_w, R.ord + t0, R.H, nt,
                   r->mode == PVT_CA_FF ? 1 : 0, R.lo, R.hi, L};
    Scope sc(ctx, PVT_K_SCORE, (double)nt * Hl, (double)nt * Hl * bpc, st, "ordered_kernel");
    launch_ordered(oa, st);
  } else if (R.band) {
    const int S = R.band_S;
    ENSURE(ctx->seg, sizeof(SegEntry) * (size_t)nt * S * KL);
    ENSURE(ctx->seg_feas, sizeof(int32_t) * (size_t)nt * S);
    const int n = R.hi - R.lo;
    // Representative rows (unsharded rounds, walked by the one-wave list walk, which maps each
    // task to its row): one list per run of equal demands instead of one per task.
    const bool reps = !R.runs.empty() && !R.full_lists;
    R.reps[lb] = reps;
    const double* dem_l = dem_w;
    const int32_t* nt_dev = nullptr;
    int nt_l = nt;
    if (reps) {                   // the rows: the runs the window spans
      const int b0 = R.runs[t0];
      R.rbase[lb] = b0;
      nt_l = R.runs[t0 + nt - 1] - b0 + 1;
      dem_l = P<double>(ctx->brdem) + (size_t)b0 * 4;
    }
    BandArgs ba{P<uint64_t>(ctx->bkey) + n, P<double>(ctx->bsa), P<uint32_t>(ctx->bstb),
                P<int32_t>(ctx->bidx) + n, n, R.lo, R.hi, P<uint8_t>(ctx->btouch),
                P<int32_t>(ctx->btlist), P<int32_t>(ctx->btcnt), r->avail, r->tiebreak, R.H, dem_l,
                nt_l, S, P<SegEntry>(ctx->seg), P<int32_t>(ctx->seg_feas), nt_dev,
                P<uint8_t>(ctx->bptouch), gate};
    {
      Scope sc(ctx, PVT_K_SCORE, (double)nt * Hl, (double)nt * Hl * bpc, st, "band_score_kernel");
      launch_band_score(ba, st);
    }
    MergeArgs ma{P<SegEntry>(ctx->seg), P<int32_t>(ctx->seg_feas), r->avail, r->zone, dem_l,
                 anc_w, R.ord + t0, R.H, nt_l, S, KL, L, nt_dev, ctx->t_merge_bitonic, gate};
    Scope sc(ctx, PVT_K_MERGE, 0, 0, st, merge_kernel_name(ma));
    launch_merge(ma, st);
  } else {
    const int S = choose_segments(Hl, nt, r->mode, ctx->score_tw, R.in_epoch, ctx->t_segments);
    ENSURE(ctx->seg, sizeof(SegEntry) * (size_t)nt * S * KL);
    ENSURE(ctx->seg_feas, sizeof(int32_t) * (size_t)nt * S);
    ScoreArgs sa{r->avail, r->zone, r->tiebreak, R.keyed ? P<double>(ctx->key) : nullptr,
                 dem_w, anc_w, P<double>(ctx->csum), P<double>(ctx->bsum), R.H, R.Z, nt, S,
                 R.lo, R.hi, P<SegEntry>(ctx->seg), P<int32_t>(ctx->seg_feas), ctx->score_tw,
                 r->mode == PVT_CA_BF ? r->rt_bw : nullptr, P<int32_t>(ctx->grp_ord) + t0};
    {
      Scope sc(ctx, PVT_K_SCORE, (double)nt * Hl, (double)nt * Hl * bpc, st, "score_kernel");
      launch_score(r->mode, sa, st);
    }
    MergeArgs ma{P<SegEntry>(ctx->seg), P<int32_t>(ctx->seg_feas), r->avail, r->zone, dem_w,
                 anc_w, R.ord + t0, R.H, nt, S, KL, L, nullptr, ctx->t_merge_bitonic};
    Scope sc(ctx, PVT_K_MERGE, 0, 0, st, merge_kernel_name(ma));
    launch_merge(ma, st);
  }
  HIPCHK(hipGetLastError());
  return PVT_OK;
}

// Launch the commit walk of tasks [t0, t0 + nt) on list buffer `lb` (inheriting n_prev hosts
// from the other buffer's walk); status -> ctx->next_host after a sync.
static int walk_launch(pvt_ctx* ctx, int t0, int nt, int lb, int n_prev) {
  RoundState& R = ctx->rs;
  const pvt_round* r = &R.r;
  hipStream_t st = ctx->stream;
  Lists L;
  lists_from(ctx, L, lb);
  int32_t* status = P<int32_t>(ctx->next);
  CommitArgs ca_{r->avail, P<double>(ctx->dem_ord) + (size_t)t0 * 4, P<double>(ctx->csum),
                 P<double>(ctx->bsum), r->zone, r->tiebreak, L, R.H, R.Z, nt, r->mode,
                 r->placement, P<int32_t>(ctx->owned[1 - lb]), n_prev, P<int32_t>(ctx->owned[lb]),
                 status, r->mode == PVT_CA_BF ? r->rt_bw : nullptr, P<int32_t>(ctx->grp_ord) + t0,
                 ctx->stamps};
  R.lw_last = r->mode == PVT_VBP_BF && ctx->lwalk && n_prev <= 2048;
  R.lw_lb = lb;
  R.lw_prev = n_prev;
  if (R.band && R.reps[lb]) {
    if (!R.lw_last) return fail(ctx, PVT_EHIP, "representative lists need the one-wave list walk");
    ca_.rowmap = P<int32_t>(ctx->brun) + t0;
    ca_.rowbase = R.rbase[lb];
    ca_.ordw = R.ord + t0;
  }
  R.lw_flag = R.lw_last;
  if (R.lw_flag) {               // the walk reports to mapped pinned words: the host polls them
    ca_.hflag = ctx->flag_hdev + 4;
    ca_.hseq = ++ctx->walk_seq;
  }
  {
    Scope sc(ctx, PVT_K_COMMIT, 0, 0, nullptr, R.lw_last ? "lwalk_kernel" : "commit_kernel");
    if (R.lw_last) launch_lwalk(ca_, st);
    else launch_commit(ca_, st);
  }
  HIPCHK(hipGetLastError());
  if (!R.lw_flag)
    HIPCHK(hipMemcpyAsync(ctx->next_host, status, sizeof(int32_t) * 2, hipMemcpyDeviceToHost, st));
  if (R.band) { R.touch_lb = lb; R.touch_status = status; }   // its hosts become touched before
                                                              // the next band score
  return PVT_OK;
}

// Window-size adaptation after a walk that advanced `adv` of `nt` tasks.
static void adapt_window(pvt_ctx* ctx, int adv, int nt) {
  RoundState& R = ctx->rs;
  if (adv < nt) {
    ctx->refills++;
    R.W = std::max(std::min(64, R.Wmax), std::min(R.Wmax, adv + adv / 2));
  } else if (nt == R.W) {
    R.W = std::min(R.Wmax, 2 * R.W);
  }
}

// The one-wave list walk could not start the window [t0, t0 + nt) (R.lw_lb, R.lw_prev): the
// list walk walks it instead; *adv = where it stopped (after a synchronisation).
static int lw_fallback(pvt_ctx* ctx, int t0, int nt, int* adv) {
  // the one-wave list walk could not start this window (its first task's list ends before
  // its bound, or too many inherited hosts): the list walk walks it, on the same lists
  RoundState& R = ctx->rs;
  const pvt_round* r = &R.r;
  if (R.reps[R.lw_lb]) {
    // representative rows: the list walk reads one list per task, so the window is scored
    // again with one (on the current state: capacities only fall, and the inherited hosts are
    // rescored as touched). The side stream's scoring shares the segment scratch: wait for it.
    if (ctx->side) HIPCHK(hipStreamSynchronize(ctx->side));
    R.full_lists = true;
    const int rc = window_lists(ctx, t0, nt, R.lw_lb, ctx->stream);
    R.full_lists = false;
    if (rc) return rc;
  }
  Lists L;
  lists_from(ctx, L, R.lw_lb);
  CommitArgs ca_{r->avail, P<double>(ctx->dem_ord) + (size_t)t0 * 4, P<double>(ctx->csum),
                 P<double>(ctx->bsum), r->zone, r->tiebreak, L, R.H, R.Z, nt, r->mode,
                 r->placement, P<int32_t>(ctx->owned[1 - R.lw_lb]), R.lw_prev,
                 P<int32_t>(ctx->owned[R.lw_lb]), P<int32_t>(ctx->next), nullptr,
                 P<int32_t>(ctx->grp_ord) + t0, ctx->stamps};
  R.lw_last = false;
  {
    Scope sc(ctx, PVT_K_COMMIT, 0, 0, nullptr, "commit_kernel");
    launch_commit(ca_, ctx->stream);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(ctx->next_host, P<int32_t>(ctx->next), sizeof(int32_t) * 2,
                        hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  *adv = ctx->next_host[0];
  return PVT_OK;
}

static int walk_status(pvt_ctx* ctx, int t0, int nt, bool inherited, int* adv) {
  if (ctx->rs.lw_flag) {
    ctx->rs.lw_flag = false;
    int rc = wait_host_flag(ctx, ctx->flag_host + 4, ctx->walk_seq, "list walk");
    if (rc) return rc;
    ctx->next_host[0] = __atomic_load_n(ctx->flag_host + 5, __ATOMIC_ACQUIRE);
    ctx->next_host[1] = __atomic_load_n(ctx->flag_host + 6, __ATOMIC_ACQUIRE);
  } else {
    HIPCHK(hipStreamSynchronize(ctx->stream));
  }
  *adv = ctx->next_host[0];
  if (*adv == 0 && ctx->rs.lw_last) {
    int rc = lw_fallback(ctx, t0, nt, adv);
    if (rc) return rc;
  }
  if (*adv == -1) return fail(ctx, PVT_EHIP, "commit walk: ring hand-off timed out at task %d", t0);
  if (*adv < 0 || *adv > nt) return fail(ctx, PVT_EHIP, "commit walk returned %d of %d", *adv, nt);
  if (*adv == 0 && !inherited) {
    if (ctx->rs.kscan && ctx->rs.kmode == 1) {   // a zero-key prefix ran dry: sort the rest
      ctx->rs.kstall = true;
      return PVT_OK;
    }
    return fail(ctx, PVT_EHIP, "commit walk made no progress at task %d", t0);
  }
  return PVT_OK;
}

// vbp first-fit and unsorted cost_aware first-fit (host index order; fit >= / strict): the
// frontier walk (pvt_zwalk.hip, keyed mode) over the first ZW_M alive hosts -- those fitting the
// smallest demand of the remaining tasks, in index order; no other host can take any of them --
// takes tasks until one fits no window host; the window is rebuilt from the current capacities
// and the walk goes on while each attempt places at least ORDERED_FRONTIER_MIN tasks, then one
// list window (which handles tasks that fit far away or nowhere) and the frontier again.
static int ordered_frontier(pvt_ctx* ctx) {
  RoundState& R = ctx->rs;
  if (!R.ofront) return PVT_OK;
  const pvt_round* r = &R.r;
  hipStream_t st = ctx->stream;
  const bool strict = r->mode == PVT_CA_FF;
  while (R.T - R.t0 >= ORDERED_FRONTIER_MIN) {
    // a bounded task prefix: its smallest demand is close to each task's own (decreasing
    // orders), so hosts filled too far for it leave the window
    const int n = std::min(R.T - R.t0, R.of_tasks);
    const double* dem = P<double>(ctx->dem_ord) + (size_t)R.t0 * 4;
    // the window comes from the first R.ofh hosts (a window of fewer than ZW_M hosts stops the
    // walk at the first task fitting none of them, which is still the answer for the tasks
    // before it); the span doubles when an attempt stops on a short window
    const int hs = std::min(R.ofh, R.H);
    {
      Scope sc(ctx, PVT_K_OTHER, 0, 0);
      launch_alive_flags(r->avail, R.H, 0, hs, dem, n, strict ? 1 : 0, P<double>(ctx->hmin),
                         P<uint8_t>(ctx->kflag), st);
      size_t tmp = ctx->ksorttmp.n;
      HIPCHK(hipcub::DeviceSelect::Flagged(P<void>(ctx->ksorttmp), tmp, P<int32_t>(ctx->kiota),
                                           P<uint8_t>(ctx->kflag), P<int32_t>(ctx->kperm),
                                           P<int32_t>(ctx->next) + 2, hs, st));
    }
    ENSURE(ctx->wres, sizeof(WinRec) * (size_t)n);
    ZwalkArgs za{r->avail, r->zone, R.H, R.Z, dem, P<int32_t>(ctx->anc_ord) + R.t0, R.ord + R.t0,
                 nullptr, nullptr, nullptr, nullptr, P<int32_t>(ctx->next), P<WinRec>(ctx->wres),
                 r->placement, nullptr, ctx->stamps, P<int32_t>(ctx->kperm), 0, 0, n, r->avail,
                 P<int32_t>(ctx->next) + 2};
    {
      Scope sc(ctx, PVT_K_COMMIT, 0, 0, nullptr, "zwalk_kernel");
      launch_zwalk_keyed(za, strict, st);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(ctx->next_host, P<int32_t>(ctx->next), sizeof(int32_t) * 3,
                          hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    const int done = ctx->next_host[0];
    if (done < 0 || done > n) return fail(ctx, PVT_EHIP, "ordered frontier walk returned %d of %d", done, n);
    ctx->n_zchains += done > 0;
    R.t0 += done;
    const bool short_window = ctx->next_host[2] < ZW_M && hs < R.H;
    if (done < n && short_window) {
      R.ofh = (int)std::min<int64_t>((int64_t)R.ofh * 2, R.H);
      if (done == 0) continue;
    }
    if (done < ORDERED_FRONTIER_MIN) break;
  }
  return PVT_OK;
}

// vbp best-fit rounds on band lists walked by the one-wave list walk, without a host round trip
// per window: up to AHEAD_MAX walks are enqueued at once, each window's size the one a run of
// complete walks takes (adapt_window), the next window's lists scored on the side stream while
// a walk runs (as place_pipelined). Walk k reads the status slot of walk k - 1 (CommitArgs::gate):
// if that one stopped early or was skipped, walk k is skipped -- and so are the scoring kernels
// of window k + 1, gated on walk k - 1 likewise -- so after a refill at most the one speculative
// window already scored is wasted, as before. Then one synchronisation reads every slot: the
// first walk that stopped early is a refill (lists from where it stopped, on the current state).
// Off by default (PVT_AHEAD=1 turns it on): measured at config 5 (rocprofv3 kernel traces of
// tools/walk_probe.py) 6.9-7.9 ms per round against 3.9-4.2 ms with a host round trip per
// window -- a third of the windows refill, and every skipped window still costs its five
// dependent launches' ~15 us gaps (two of them across streams), more than the round trips saved.
static int place_ahead(pvt_ctx* ctx) {
  RoundState& R = ctx->rs;
  int rc, nt = 0;
  if ((rc = round_next_window(ctx, &nt))) return rc;
  if (nt == 0) return PVT_OK;
  ENSURE(ctx->wslot, sizeof(int32_t) * 4 * AHEAD_MAX);
  int32_t* slots = P<int32_t>(ctx->wslot);
  const int32_t* hslots = ctx->next_host + 4;
  int t0 = R.t0, lb = 0, n_prev = 0;
  bool inherited = false;
  if ((rc = window_lists(ctx, t0, nt, lb, ctx->stream))) return rc;
  struct Win { int t0, nt, lb; };
  for (;;) {
    Win q[AHEAD_MAX];
    int nq = 0, W = R.W;
    Win nx{0, 0, 0};                          // the window after the last enqueued walk
    for (;;) {
      const int32_t* gate = nq > 0 ? slots + 4 * (nq - 1) : nullptr;
      const int nt0 = t0 + nt;
      if (nt == W) W = std::min(R.Wmax, 2 * W);   // (adapt_window after a complete walk)
      const int nnt = nt0 < R.T ? std::min(W, R.T - nt0) : 0;
      flush_touched(ctx);                     // the walk before's hosts (none if it was skipped)
      if (nnt > 0) HIPCHK(hipEventRecord(ctx->ev_walk, ctx->stream));
      {
        Lists L;
        lists_from(ctx, L, lb);
        const pvt_round* r = &R.r;
        int32_t* slot = slots + 4 * nq;
        CommitArgs ca_{r->avail, P<double>(ctx->dem_ord) + (size_t)t0 * 4, P<double>(ctx->csum),
                       P<double>(ctx->bsum), r->zone, r->tiebreak, L, R.H, R.Z, nt, r->mode,
                       r->placement, P<int32_t>(ctx->owned[1 - lb]), nq == 0 ? n_prev : 0,
                       P<int32_t>(ctx->owned[lb]), slot, nullptr, P<int32_t>(ctx->grp_ord) + t0,
                       ctx->stamps};
        if (R.reps[lb]) {
          ca_.rowmap = P<int32_t>(ctx->brun) + t0;
          ca_.rowbase = R.rbase[lb];
          ca_.ordw = R.ord + t0;
        }
        ca_.gate = gate;
        ca_.ahead = 1;
        {
          Scope sc(ctx, PVT_K_COMMIT, 0, 0, nullptr, "lwalk_kernel");
          launch_lwalk(ca_, ctx->stream);
        }
        HIPCHK(hipGetLastError());
        R.touch_lb = lb;
        R.touch_status = slot;
      }
      q[nq++] = {t0, nt, lb};
      if (nnt > 0) {
        HIPCHK(hipStreamWaitEvent(ctx->side, ctx->ev_walk, 0));
        if ((rc = window_lists(ctx, nt0, nnt, 1 - lb, ctx->side, gate))) return rc;
        HIPCHK(hipEventRecord(ctx->ev_lists, ctx->side));
        HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->ev_lists, 0));
      }
      nx = {nt0, nnt, 1 - lb};
      if (nnt == 0 || nq == AHEAD_MAX) break;
      t0 = nt0; nt = nnt; lb = 1 - lb;
    }
    HIPCHK(hipMemcpyAsync(ctx->next_host + 4, slots, sizeof(int32_t) * 4 * nq, hipMemcpyDeviceToHost,
                          ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    int j = 0, adv = 0;
    for (; j < nq; j++) {
      adv = hslots[4 * j];
      if (hslots[4 * j + 3] != 0 || adv < 0 || adv > q[j].nt)
        return fail(ctx, PVT_EHIP, "list walk %d of %d returned %d of %d (skipped %d)", j, nq, adv,
                    q[j].nt, hslots[4 * j + 3]);
      if (adv < q[j].nt) break;
      adapt_window(ctx, adv, q[j].nt);
    }
    if (j == nq) {                            // every walk took its whole window
      if (nx.nt == 0) { R.t0 = R.T; break; }
      n_prev = hslots[4 * (nq - 1) + 1];
      t0 = nx.t0; nt = nx.nt; lb = nx.lb;
      inherited = true;
      continue;
    }
    // walk j stopped early: the walks after it were skipped, as were the scorings after the
    // speculative one (discarded here)
    if (adv == 0) {
      R.lw_lb = q[j].lb;
      R.lw_prev = j == 0 ? n_prev : hslots[4 * (j - 1) + 1];
      if ((rc = lw_fallback(ctx, q[j].t0, q[j].nt, &adv))) return rc;
      R.touch_lb = q[j].lb;
      R.touch_status = P<int32_t>(ctx->next);
      if (adv == -1) return fail(ctx, PVT_EHIP, "commit walk: ring hand-off timed out at task %d", q[j].t0);
      if (adv < 0 || adv > q[j].nt) return fail(ctx, PVT_EHIP, "commit walk returned %d of %d", adv, q[j].nt);
      if (adv == 0 && !(inherited || j > 0))
        return fail(ctx, PVT_EHIP, "commit walk made no progress at task %d", q[j].t0);
    }
    adapt_window(ctx, adv, q[j].nt);
    HIPCHK(hipStreamSynchronize(ctx->side));
    flush_touched(ctx);
    R.t0 = q[j].t0 + adv;
    if ((rc = round_next_window(ctx, &nt))) return rc;
    if (nt == 0) break;
    t0 = R.t0; lb = 0; n_prev = 0; inherited = false;
    if ((rc = window_lists(ctx, t0, nt, lb, ctx->stream))) return rc;
  }
  flush_touched(ctx);
  return PVT_OK;
}

// pvt_place for the list policies. While window k is walked on the caller's stream, the side
// stream scores window k+1 on the capacities as they stand (the walk of k-1 is complete; the
// walk of k is in flight): an event recorded just before walk k releases it. The side stream
// runs on all but a few CUs (create_side_stream), so the score grid never holds back the walk,
// which needs a whole CU's LDS. Hosts window k commits to are the only ones whose list entries
// can be stale, so walk k+1 inherits them as touched (pvt_walk.hip) and stays exact. A walk that
// stops early (refill) discards the speculative lists; keyed first-fit recomputes its frozen
// key at a group start, so the pipeline drains at group boundaries.
static int place_pipelined(pvt_ctx* ctx) {
  RoundState& R = ctx->rs;
  int rc, nt = 0;
  if (R.band && ctx->lwalk && ctx->ahead && ctx->pipeline && !R.sharded && !R.ofront && !R.keyed)
    return place_ahead(ctx);
  if ((rc = ordered_frontier(ctx))) return rc;
  if ((rc = round_next_window(ctx, &nt))) return rc;
  if (nt == 0) return PVT_OK;
  int lb = 0, t0 = R.t0;
  if ((rc = window_lists(ctx, t0, nt, lb, ctx->stream))) return rc;
  int n_prev = 0;
  bool inherited = false;
  for (;;) {
    // Walk k, and beside it window k+1 (same group) scored on the state walk k-1 left.
    const int nt0 = t0 + nt, ge = group_end(R, t0);
    // (ordered frontier rounds: no speculative window; the frontier walk is tried after each)
    const int nnt = (ctx->pipeline && nt0 < ge && !R.ofront) ? std::min(R.W, ge - nt0) : 0;
    flush_touched(ctx);   // the previous walk's hosts, seen by the score pass launched next
    if (nnt > 0) HIPCHK(hipEventRecord(ctx->ev_walk, ctx->stream));
    if ((rc = walk_launch(ctx, t0, nt, lb, n_prev))) return rc;
    if (nnt > 0) {
      HIPCHK(hipStreamWaitEvent(ctx->side, ctx->ev_walk, 0));
      if ((rc = window_lists(ctx, nt0, nnt, 1 - lb, ctx->side))) return rc;
      HIPCHK(hipEventRecord(ctx->ev_lists, ctx->side));
    }
    int adv = 0;
    if ((rc = walk_status(ctx, t0, nt, inherited, &adv))) return rc;
    const int n_own = ctx->next_host[1];
    adapt_window(ctx, adv, nt);
    if (adv == nt && nnt > 0) {                 // take the speculative window
      HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->ev_lists, 0));
      t0 = nt0; nt = nnt; lb = 1 - lb; n_prev = n_own; inherited = true;
      continue;
    }
    if (nnt > 0) HIPCHK(hipStreamSynchronize(ctx->side));   // discard the speculation
    flush_touched(ctx);
    R.t0 = t0 + adv;
    if ((rc = ordered_frontier(ctx))) return rc;
    if ((rc = round_next_window(ctx, &nt))) return rc;
    if (nt == 0) break;
    t0 = R.t0; lb = 0; n_prev = 0; inherited = false;
    if ((rc = window_lists(ctx, t0, nt, lb, ctx->stream))) return rc;
  }
  return PVT_OK;
}

// ---------------------------------------------------------------- group-parallel epochs
// Zones joined by zero egress cost (csum = 0) form one component: a group's winners are the
// lowest-index fitting hosts of its anchor's component (score 0), so two groups anchored in one
// component compete for the same hosts and an epoch never holds both (R.ecomp: zone -> root).
static int zero_cost_components(pvt_ctx* ctx) {
  RoundState& R = ctx->rs;
  const pvt_round* r = &R.r;
  const int Z = R.Z;
  std::vector<double> cost((size_t)Z * Z);
  if (R.ginfo && R.cost_host.size() == cost.size()) {
    cost = R.cost_host;
  } else {
    HIPCHK(hipMemcpyAsync(cost.data(), r->cost, sizeof(double) * Z * Z, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
  }
  R.ecomp.resize(Z);
  for (int z = 0; z < Z; z++) R.ecomp[z] = z;
  auto root = [&](int z) { while (R.ecomp[z] != z) z = R.ecomp[z] = R.ecomp[R.ecomp[z]]; return z; };
  const int plan = ctx->t_epoch_plan;   // (PVT_EPOCH_PLAN=0: distinct zones only)
  for (int a = 0; a < Z && plan; a++)
    for (int z = 0; z < Z; z++)
      if (cost[(size_t)a * Z + z] + cost[(size_t)z * Z + a] == 0.0) R.ecomp[root(a)] = root(z);
  for (int z = 0; z < Z; z++) R.ecomp[z] = root(z);
  return PVT_OK;
}

// cost_aware best-fit rounds of several groups (pvt_epoch.hip). The groups in processing
// order, from the caller's task_group / group_anchor (a group's tasks are contiguous).
static int epoch_groups(pvt_ctx* ctx) {
  RoundState& R = ctx->rs;
  const pvt_round* r = &R.r;
  R.egs.clear();
  R.ega.clear();
  const int T = R.T;
  if (!ctx->epochs || r->mode != PVT_CA_BF || !r->task_group || r->n_groups < 2 || T < 2) return PVT_OK;
  hipStream_t st = ctx->stream;
  int rc;
  std::vector<int> cnt(r->n_groups, 0);
  std::vector<int32_t> ga;
  if (R.ginfo) {                              // copied by build_order
    for (int g = 0; g < r->n_groups; g++) cnt[g] = R.gcnt[g];
    ga = R.ga_host;
  } else {
    std::vector<int32_t> tg(T);
    ga.resize(r->n_groups);
    HIPCHK(hipMemcpyAsync(tg.data(), r->task_group, sizeof(int32_t) * T, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(ga.data(), r->group_anchor, sizeof(int32_t) * r->n_groups,
                          hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    for (int t = 0; t < T; t++) {
      if (tg[t] < 0 || tg[t] >= r->n_groups) return fail(ctx, PVT_EINVAL, "task_group out of range");
      cnt[tg[t]]++;
    }
  }
  int off = 0, ng = 0;
  for (int g = 0; g < r->n_groups; g++) {
    if (cnt[g] == 0) continue;
    R.egs.push_back(off);
    R.ega.push_back(ga[g]);
    off += cnt[g];
    ng++;
  }
  R.egs.push_back(T);
  if ((rc = zero_cost_components(ctx))) return rc;
  // worth it when groups are many and short (a group longer than a walk's window is walked in
  // sequential epochs of one segment, without the score / walk pipeline of place_pipelined)
  if (ng < 2 || T > ng * MAX_WINDOW) { R.egs.clear(); R.ega.clear(); }
  return PVT_OK;
}

static void epoch_plan(const RoundState& R, int t0, EpochPlan& P, bool whole = false) {
  P.off.assign(1, 0);
  P.chain.clear(); P.cstart.clear(); P.segs.clear(); P.len.clear();
  size_t g = 0;
  while (g + 1 < R.egs.size() && R.egs[g + 1] <= t0) g++;
  std::vector<int> chain_of(R.ecomp.size() + 1, -1);
  int t = t0;
  while (t < R.T && (int)P.chain.size() < EPOCH_SEGS) {
    const int ge = R.egs[g + 1];
    const int z = R.ega[g];
    const int comp = (z >= 0 && z < (int)R.ecomp.size()) ? R.ecomp[z] : (int)R.ecomp.size();
    int c = chain_of[comp];
    if (c < 0) {
      c = chain_of[comp] = (int)P.segs.size();
      P.segs.emplace_back();
      P.len.push_back(0);
    }
    const int take = std::min({ge - t, CHAIN_MAX - P.len[c], t0 + EPOCH_MAX - t});
    if (take <= 0 || (whole && take < ge - t)) {
      if (P.len[c] == 0) { P.segs.pop_back(); P.len.pop_back(); }   // (a chain opened for it)
      break;
    }
    P.segs[c].push_back((int)P.chain.size());
    P.chain.push_back(c);
    P.cstart.push_back(P.len[c]);
    P.len[c] += take;
    t += take;
    P.off.push_back(t - t0);
    if (t < ge) break;
    g++;
  }
}

// The epoch's chain tables to the device (one upload): segment offsets / chains / chain-local
// starts, per chain its task range in cmap and its segments' chain-local starts.
static int upload_chain_tables(pvt_ctx* ctx, const EpochPlan& E) {
  int32_t* host = ctx->ep_host;
  const int nseg = (int)E.chain.size(), nch = (int)E.segs.size();
  for (int k = 0; k <= nseg; k++) host[EP_SEG_OFF + k] = E.off[k];
  for (int k = 0; k < nseg; k++) { host[EP_SEG_CHAIN + k] = E.chain[k]; host[EP_SEG_CSTART + k] = E.cstart[k]; }
  int nm = 0, ns = 0;
  for (int c = 0; c < nch; c++) {
    host[EP_COFF + c] = nm;
    host[EP_CSOFF + c] = ns;
    for (int sg : E.segs[c]) {
      host[EP_CSEG + ns++] = E.cstart[sg];
      for (int w = E.off[sg]; w < E.off[sg + 1]; w++) host[EP_CMAP + nm++] = w;
    }
  }
  host[EP_COFF + nch] = nm;
  host[EP_CSOFF + nch] = ns;
  launch_upload(ctx->ep_hdev, ctx->ep_dev.p, sizeof(int32_t) * (EP_CMAP + nm), ctx->stream);
  HIPCHK(hipGetLastError());
  return PVT_OK;
}

// The same tables by value for the frontier walk (ChainTab: no upload launch); false when the
// epoch does not fit them (the caller uploads instead).
static_assert(EPOCH_SEGS == CT_SEGS, "chain tables by value hold every epoch segment");
static bool chain_tab(pvt_ctx* ctx, const EpochPlan& E, ChainTab& t) {
  const int nseg = (int)E.chain.size(), nch = (int)E.segs.size();
  if (nseg < 1 || nseg > CT_SEGS || nch < 1 || nch > CT_SEGS) return false;
  for (int c = 0; c < nch; c++)
    if (E.len[c] > CHAIN_MAX) return false;
  int32_t* dev = P<int32_t>(ctx->ep_dev);
  t.nseg = nseg;
  t.nch = nch;
  for (int k = 0; k <= nseg; k++) t.seg_off[k] = E.off[k];
  for (int k = 0; k < nseg; k++) { t.seg_chain[k] = E.chain[k]; t.seg_cstart[k] = E.cstart[k]; }
  int nm = 0, ns = 0;
  for (int c = 0; c < nch; c++) {
    t.coff[c] = nm;
    t.csoff[c] = ns;
    for (int sg : E.segs[c]) t.csegid[ns++] = sg;
    nm += E.len[c];
  }
  t.coff[nch] = nm;
  t.csoff[nch] = ns;
  t.o_seg_off = dev + EP_SEG_OFF;
  t.o_seg_chain = dev + EP_SEG_CHAIN;
  t.o_seg_cstart = dev + EP_SEG_CSTART;
  t.o_coff = dev + EP_COFF;
  return true;
}

// cost_aware first-fit with sort_hosts (cost_aware.py:99-127): an epoch of WHOLE groups from
// the group start R.t0, chains of zero-cost components walked side by side by the first-fit
// zero-key chain walk (pvt_zwalk.hip, FF). Every task it proves takes the lowest-index strictly
// fitting host of its anchor's zero-cost zones -- the first host of the frozen key order -- and
// chains of different components touch disjoint hosts that are never zero-key for another
// chain's anchors, so no pair validation is needed. Groups are accepted whole, in order, up to
// the first one a chain did not complete (the keyed path then takes that group from its start,
// computing its frozen key on the capacities at the group start, as the reference does).
static int ff_epoch(pvt_ctx* ctx, int* adv_out) {
  RoundState& R = ctx->rs;
  const pvt_round* r = &R.r;
  hipStream_t st = ctx->stream;
  *adv_out = 0;
  const int t0 = R.t0;
  EpochPlan E;
  epoch_plan(R, t0, E, true);
  const int nseg = (int)E.chain.size(), nch = (int)E.segs.size();
  if (nseg == 0 || nch == 0) return PVT_OK;
  const int nt = E.off.back();
  ENSURE(ctx->ep_dev, sizeof(int32_t) * EP_WORDS);
  ENSURE(ctx->wres, sizeof(WinRec) * (size_t)EPOCH_MAX);
  ENSURE(ctx->hmin, sizeof(double) * 4 * ZW_MIN_PARTS);
  int32_t* dev = P<int32_t>(ctx->ep_dev);
  int32_t* host = ctx->ep_host;
  int rc;
  {
    Scope sc(ctx, PVT_K_OTHER, 0, 0);
    launch_host_absmax(r->avail, R.H, 0, R.H, P<double>(ctx->hmin), st);
  }
  ZwalkArgs za{r->avail, r->zone, R.H, R.Z, P<double>(ctx->dem_ord) + (size_t)t0 * 4,
               P<int32_t>(ctx->anc_ord) + t0, R.ord + t0, P<double>(ctx->csum),
               P<double>(ctx->bsum), dev + EP_COFF, dev + EP_CMAP, dev + EP_STATUS,
               P<WinRec>(ctx->wres), r->placement, P<double>(ctx->hmin), ctx->stamps,
               nullptr, 0, 0, 0, nullptr, nullptr, nullptr, dev + EP_CSOFF, dev + EP_CSEG};
  if (!(ctx->t_chain_tab && chain_tab(ctx, E, za.tab)) && (rc = upload_chain_tables(ctx, E))) return rc;
  {
    Scope sc(ctx, PVT_K_COMMIT, 0, 0, nullptr, "zwalk_kernel");
    launch_zwalk_ff(za, nch, st);
  }
  EpochArgs ea{P<double>(ctx->dem_ord) + (size_t)t0 * 4, P<int32_t>(ctx->anc_ord) + t0,
               P<double>(ctx->csum), P<double>(ctx->bsum), r->zone, dev + EP_SEG_OFF,
               dev + EP_SEG_CHAIN, dev + EP_SEG_CSTART, dev + EP_STATUS, P<WinRec>(ctx->wres),
               r->avail, R.H, R.Z, nt, nseg, dev + EP_BAD, nullptr, P<int32_t>(ctx->grp_ord) + t0, 1};
  {
    Scope sc(ctx, PVT_K_OTHER, 0, 0);
    launch_epoch_final(ea, st);
    launch_epoch_accept_apply(ea, dev + EP_RES, nch, st, ctx->ep_hdev + EP_STATUS,
                              EP_WORDS - EP_STATUS);   // (readback: mapped)
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(st));
  ctx->n_epochs++;
  ctx->n_segs += nseg;
  int proven = 0;
  for (int c = 0; c < nch; c++) proven += host[EP_STATUS + 2 * c] == E.len[c];
  ctx->n_zchains += proven;
  ctx->n_longest += *std::max_element(E.len.begin(), E.len.end());
  ctx->n_rejected += host[EP_RES + 3];
  const int adv = host[EP_RES + 1];
  if (adv < 0 || adv > nt) return fail(ctx, PVT_EHIP, "first-fit epoch returned %d of %d tasks", adv, nt);
  *adv_out = adv;
  return PVT_OK;
}

// A frontier-walked epoch's verdict (validation, accepted prefix and its apply ran on the
// device; ctx->ep_host holds the readback): chains left unproven, and the tasks accepted.
static int epoch_frontier_verdict(pvt_ctx* ctx, const EpochPlan& E, int t0, int* need_out, int* adv_out) {
  const int32_t* host = ctx->ep_host;
  const int nch = (int)E.segs.size();
  int need = 0;
  for (int c = 0; c < nch; c++) need += host[EP_STATUS + 2 * c] != E.len[c];
  ctx->n_zchains += nch - need;
  ctx->n_longest += *std::max_element(E.len.begin(), E.len.end());
  if (host[EP_RES + 4])
    return fail(ctx, PVT_EHIP, "commit walk: ring hand-off timed out (epoch at task %d)", t0);
  const int adv = host[EP_RES + 1];
  // (a segment cut short here is a frontier-walk fallback, not a list refill: the chains the
  // walk could not prove are walked with lists next; the tasks it proved are accepted)
  ctx->n_rejected += host[EP_RES + 3];
  if (adv <= 0 && !need) return fail(ctx, PVT_EHIP, "epoch made no progress at task %d", t0);
  *need_out = need;
  *adv_out = adv;
  return PVT_OK;
}

static int place_epochs(pvt_ctx* ctx) {
  RoundState& R = ctx->rs;
  const pvt_round* r = &R.r;
  hipStream_t st = ctx->stream;
  ENSURE(ctx->ep_dev, sizeof(int32_t) * EP_WORDS);
  ENSURE(ctx->wres, sizeof(WinRec) * (size_t)EPOCH_MAX);
  ENSURE(ctx->owned[0], sizeof(int32_t) * (size_t)CHAIN_MAX);
  ENSURE(ctx->l_e[0], sizeof(ListEntry) * (size_t)EPOCH_MAX * LMAX);
  ENSURE(ctx->l_ids[0], sizeof(int32_t) * (size_t)EPOCH_MAX * LMAX);
  ENSURE(ctx->l_t[0], sizeof(TaskRec) * (size_t)EPOCH_MAX);
  int32_t* dev = P<int32_t>(ctx->ep_dev);
  int32_t* host = ctx->ep_host;
  EpochPlan E;
  int t0 = 0, rc;
  bool force_lists = false;       // the last epoch's frontier walk left chains unproven
  bool big = false;               // ... because a chain outgrew its window: retry with ZW_MBIG
  int big_t0 = -1;                //   (at most once per epoch start)
  R.in_epoch = true;
  struct Reset { bool& f; ~Reset() { f = false; } } reset_{R.in_epoch};
  const bool zw_possible = ctx->zwalk && !r->rt_bw && R.Z <= ZMAX;
  while (t0 < R.T) {
    // the frontier walk's host minima (certificate 2) depend only on the epoch's start state:
    // reduced while the host plans the epoch
    if (zw_possible && !force_lists && !(R.hmin_pre && t0 == 0)) {
      ENSURE(ctx->hmin, sizeof(double) * 4 * ZW_MIN_PARTS);
      Scope sc(ctx, PVT_K_OTHER, 0, 0);
      launch_host_min(r->avail, R.H, 0, R.H, P<double>(ctx->hmin), st);
    }
    R.hmin_pre = false;
    epoch_plan(R, t0, E);
    const int nseg = (int)E.chain.size(), nch = (int)E.segs.size(), nt = E.off.back();
    ctx->n_epochs++;
    ctx->n_segs += nseg;
    // chains the zero-cost frontier walk can prove need no candidate lists (pvt_zwalk.hip);
    // the lists are scored only for the others
    const bool zw = ctx->zwalk && nch > 1 && !r->rt_bw && R.Z <= ZMAX && !force_lists;
    force_lists = false;
    if (!zw && (rc = window_lists(ctx, t0, nt, 0, st))) return rc;
    Lists L;
    lists_from(ctx, L, 0);
    if (nch == 1) {                           // one chain: the plain walk (writes avail)
      if ((rc = walk_launch(ctx, t0, nt, 0, 0))) return rc;
      int adv = 0;
      if ((rc = walk_status(ctx, t0, nt, false, &adv))) return rc;
      if (adv < nt) ctx->refills++;
      t0 += adv;
      continue;
    }
    // (the frontier walk takes the chain tables by value: no upload)
    ChainTab tab{};
    const bool tabv = zw && ctx->t_chain_tab && chain_tab(ctx, E, tab);
    if (!tabv && (rc = upload_chain_tables(ctx, E))) return rc;
    // (the rejection flags are zeroed by epoch_final_kernel, launched before every validation)
    int need = nch;                           // chains left to the list walk
    EpochArgs ea{P<double>(ctx->dem_ord) + (size_t)t0 * 4, P<int32_t>(ctx->anc_ord) + t0,
                 P<double>(ctx->csum), P<double>(ctx->bsum), r->zone, dev + EP_SEG_OFF,
                 dev + EP_SEG_CHAIN, dev + EP_SEG_CSTART, dev + EP_STATUS, P<WinRec>(ctx->wres),
                 r->avail, R.H, R.Z, nt, nseg, dev + EP_BAD, r->rt_bw, P<int32_t>(ctx->grp_ord) + t0};
    auto validate_and_read = [&]() -> int {
      {
        Scope sc(ctx, PVT_K_OTHER, 0, 0);
        launch_epoch_validate(ea, st);
      }
      HIPCHK(hipGetLastError());
      HIPCHK(hipMemcpyAsync(host + EP_STATUS, dev + EP_STATUS, sizeof(int32_t) * (EP_WORDS - EP_STATUS),
                            hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      return PVT_OK;
    };
    if (zw) {
      ENSURE(ctx->cmax, sizeof(double) * 4 * EPOCH_SEGS);
      ZwalkArgs za{r->avail, r->zone, R.H, R.Z, P<double>(ctx->dem_ord) + (size_t)t0 * 4,
                   P<int32_t>(ctx->anc_ord) + t0, R.ord + t0, P<double>(ctx->csum),
                   P<double>(ctx->bsum), dev + EP_COFF, dev + EP_CMAP, dev + EP_STATUS,
                   P<WinRec>(ctx->wres), r->placement, P<double>(ctx->hmin), ctx->stamps,
                   nullptr, 0, 0, 0, nullptr, nullptr, nullptr, dev + EP_CSOFF, dev + EP_CSEG,
                   P<double>(ctx->cmax)};
      // (the first epoch starts from the snapshot the grouped order's launch built its windows from)
      if (R.zpre && t0 == 0 && !big) za.zpre = P<ZoneWindows>(ctx->zwin);
      if (tabv) za.tab = tab;
      R.zpre = false;
      ea.cmax = P<double>(ctx->cmax);
      ea.coff = dev + EP_COFF;
      ea.nch = nch;
      ea.safe = dev + EP_SAFE;
      {
        Scope sc(ctx, PVT_K_COMMIT, 0, 0, nullptr, "zwalk_kernel");
        if (big) launch_zwalk_big(za, nch, st);
        else launch_zwalk(za, nch, st);
      }
      const bool was_big = big;
      big = false;
      HIPCHK(hipGetLastError());
      // validation, the accepted prefix and its apply all on the device, then one readback. A
      // chain the frontier walk could not prove is not accepted past its first segment; the
      // next epoch then walks its chains with candidate lists (force_lists) -- or, when a chain
      // only ran out of window hosts, once more with the large window.
      {
        Scope sc(ctx, PVT_K_OTHER, 0, 0);
        launch_epoch_validate(ea, st);
        launch_epoch_accept_apply(ea, dev + EP_RES, nch, st, ctx->ep_hdev + EP_STATUS,
                                  EP_WORDS - EP_STATUS);   // (readback: mapped)
      }
      HIPCHK(hipGetLastError());
      HIPCHK(hipStreamSynchronize(st));
      int adv = 0;
      if ((rc = epoch_frontier_verdict(ctx, E, t0, &need, &adv))) return rc;
      if (need && adv < nt) {
        bool exhausted = false;
        for (int c = 0; c < nch; c++) exhausted |= host[EP_STATUS + 2 * c + 1] == 2;
        if (exhausted && !was_big && big_t0 != t0 + adv) {
          big = true;
          big_t0 = t0 + adv;
        } else {
          force_lists = true;
        }
      }
      t0 += adv;
      continue;
    }
    ctx->n_gchains += need;
    ctx->n_longest += *std::max_element(E.len.begin(), E.len.end());
    CommitArgs ca_{r->avail, P<double>(ctx->dem_ord) + (size_t)t0 * 4, P<double>(ctx->csum),
                   P<double>(ctx->bsum), r->zone, r->tiebreak, L, R.H, R.Z, nt, r->mode,
                   r->placement, nullptr, 0, P<int32_t>(ctx->owned[0]), dev + EP_STATUS,
                   r->rt_bw, P<int32_t>(ctx->grp_ord) + t0, ctx->stamps, dev + EP_COFF, dev + EP_CMAP, dev + EP_CSOFF, dev + EP_CSEG,
                   P<WinRec>(ctx->wres), zw ? 1 : 0};
    if (need) {
      {
        Scope sc(ctx, PVT_K_COMMIT, 0, 0, nullptr, "commit_kernel");
        launch_commit_chains(ca_, nch, st);
      }
      if ((rc = validate_and_read())) return rc;
    }
    // the exact prefix: segments before the first rejected one, up to and including the first
    // that its chain did not finish (its walked tasks are exact; the next epoch starts there)
    for (int c = 0; c < nch; c++)
      if (host[EP_STATUS + 2 * c] == -1)
        return fail(ctx, PVT_EHIP, "commit walk: ring hand-off timed out (epoch at task %d)", t0);
    int acc = 0, next = t0;
    for (int j = 0; j < nseg; j++) {
      const int len = E.off[j + 1] - E.off[j];
      const int adv = std::max(0, std::min(len, host[EP_STATUS + 2 * E.chain[j]] - E.cstart[j]));
      if (j > 0 && host[EP_BAD + j]) { ctx->n_rejected += nseg - j; break; }
      acc = j + 1;
      next = t0 + E.off[j] + adv;
      if (adv < len) { ctx->refills++; ctx->n_rejected += nseg - j - 1; break; }
    }
    if (next == t0) return fail(ctx, PVT_EHIP, "epoch made no progress at task %d", t0);
    {
      Scope sc(ctx, PVT_K_OTHER, 0, 0);
      launch_epoch_apply(ea, acc, nch, st);
    }
    HIPCHK(hipGetLastError());
    t0 = next;
  }
  return PVT_OK;
}

// ---------------------------------------------------------------- resident rounds / batches
static bool resident_fits(const pvt_round* r, int max_hosts) {
  return r->n_hosts <= std::min(max_hosts, (int)PVT_RESIDENT_MAX_HOSTS) &&
         r->n_tasks <= PVT_RESIDENT_MAX_TASKS;
}

template <class T>
static int ensure_pinned_array(pvt_ctx* ctx, T*& p, size_t& cap, size_t n) {
  if (cap >= n) return PVT_OK;
  const size_t want = std::max(n, cap * 3 / 2);
  if (p) (void)hipHostFree(p);
  p = nullptr;
  cap = 0;
  if (hipHostMalloc((void**)&p, sizeof(T) * want) != hipSuccess) {
    p = nullptr;
    return fail(ctx, PVT_ENOMEM, "hipHostMalloc(%zu) failed", sizeof(T) * want);
  }
  cap = want;
  return PVT_OK;
}

// desc_dev: the rounds' descriptors already on the device (pvt_place_host's staging, MT states
// at mt_dev): nothing is copied and nothing waited for here; the caller copies back and syncs.
// mt_dev alone (pvt_place_batch_mt): the rounds' MT19937 states live on the device, [n][625].
static int place_resident(pvt_ctx* ctx, const pvt_round* rounds, int n,
                          const void* desc_dev = nullptr, uint32_t* mt_dev = nullptr) {
  const int mode = rounds[0].mode;
  int maxH = 1, maxT = 1, maxZ = 1;
  for (int i = 0; i < n; i++) {
    const pvt_round* r = &rounds[i];
    int rc = check_round(ctx, r);
    if (rc) return rc;
    if (r->mode != mode) return fail(ctx, PVT_EINVAL, "batch round %d: mode %d != %d", i, r->mode, mode);
    if (!resident_fits(r, PVT_RESIDENT_MAX_HOSTS))
      return fail(ctx, PVT_EUNSUPPORTED, "batch round %d: H=%d T=%d exceeds the resident limits (%d, %d)",
                  i, r->n_hosts, r->n_tasks, PVT_RESIDENT_MAX_HOSTS, PVT_RESIDENT_MAX_TASKS);
    maxH = std::max(maxH, r->n_hosts);
    maxT = std::max(maxT, r->n_tasks);
    maxZ = std::max(maxZ, r->n_zones);
  }
  HIPCHK(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  int waves = ctx->res_waves, hpl = 1;
  resident_shape(maxH, &waves, &hpl);
  int tpad = 64;
  while (tpad < maxT) tpad <<= 1;
  const int rwalk = ctx->rwalk && maxH <= RW_MAXH ? ctx->rwalk : 0;
  double cand = 0.0, bytes = 0.0;
  for (int i = 0; i < n; i++) {
    const double c = (double)rounds[i].n_tasks * rounds[i].n_hosts;
    cand += c;
    bytes += c * bytes_per_candidate(mode);
  }
  if (desc_dev) {
    ResidentArgs ra{desc_dev, mt_dev, maxZ, tpad, ctx->stamps, rwalk};
    {
      Scope sc(ctx, PVT_K_SCORE, cand, bytes, nullptr, "resident_kernel");
      launch_resident(mode, waves, hpl, n, ra, st);
    }
    HIPCHK(hipGetLastError());
    ctx->windows = n;
    ctx->refills = 0;
    return PVT_OK;
  }
  int rc;
  // the staged descriptors (and MT states) reach the device by an upload kernel reading their
  // mapped pages when it runs: a new batch waits until the previous batch's upload has run
  if (ctx->rstage_busy) HIPCHK(hipEventSynchronize(ctx->ev_rstage));
  ctx->rstage_busy = false;
  if ((rc = ensure_pinned_array(ctx, ctx->rstage, ctx->rstage_cap, (size_t)n))) return rc;
  std::memcpy(ctx->rstage, rounds, sizeof(pvt_round) * n);
  ENSURE(ctx->rdesc, sizeof(pvt_round) * (size_t)n + 16);   // (+16: the upload's rounding)
  uint32_t* mt = nullptr;
  const bool host_mt = mode == PVT_OPP && !mt_dev;
  if (mode == PVT_OPP && mt_dev) {
    mt = mt_dev;
    for (int i = 0; i < n; i++) ctx->rstage[i].mt_state = mt + (size_t)i * 625;
  } else if (host_mt) {
    ENSURE(ctx->rmt, sizeof(uint32_t) * 625 * (size_t)n + 16);
    mt = P<uint32_t>(ctx->rmt);
    if ((rc = ensure_pinned_array(ctx, ctx->rmt_host, ctx->rmt_cap, (size_t)n * 625))) return rc;
    for (int i = 0; i < n; i++) {
      std::memcpy(ctx->rmt_host + (size_t)i * 625, rounds[i].mt_state, sizeof(uint32_t) * 625);
      ctx->rstage[i].mt_state = mt + (size_t)i * 625;   // the device copy the kernel draws from
    }
    void* dmt = nullptr;
    HIPCHK(hipHostGetDevicePointer(&dmt, ctx->rmt_host, 0));
    launch_upload(dmt, mt, sizeof(uint32_t) * 625 * n, st);
  }
  {
    void* dst = nullptr;
    HIPCHK(hipHostGetDevicePointer(&dst, ctx->rstage, 0));
    launch_upload(dst, ctx->rdesc.p, sizeof(pvt_round) * n, st);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(ctx->ev_rstage, st));
  ctx->rstage_busy = true;
  ResidentArgs ra{ctx->rdesc.p, mt, maxZ, tpad, ctx->stamps, rwalk};
  {
    Scope sc(ctx, PVT_K_SCORE, cand, bytes, nullptr, "resident_kernel");
    launch_resident(mode, waves, hpl, n, ra, st);
  }
  HIPCHK(hipGetLastError());
  if (host_mt)
    HIPCHK(hipMemcpyAsync(ctx->rmt_host, mt, sizeof(uint32_t) * 625 * n, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (host_mt)
    for (int i = 0; i < n; i++)
      std::memcpy(rounds[i].mt_state, ctx->rmt_host + (size_t)i * 625, sizeof(uint32_t) * 625);
  ctx->windows = n;
  ctx->refills = 0;
  return PVT_OK;
}

extern "C" int pvt_place_batch(pvt_ctx* ctx, const pvt_round* rounds, int32_t n_rounds) {
  if (!ctx) return PVT_EINVAL;
  if (n_rounds < 0 || (n_rounds > 0 && !rounds)) return fail(ctx, PVT_EINVAL, "bad batch (%d rounds)", n_rounds);
  ctx->rs.active = false;
  if (n_rounds == 0) return PVT_OK;
  return place_resident(ctx, rounds, n_rounds);
}

extern "C" int pvt_place_batch_mt(pvt_ctx* ctx, const pvt_round* rounds, int32_t n_rounds,
                                  uint32_t* mt_dev) {
  if (!ctx) return PVT_EINVAL;
  if (n_rounds < 0 || (n_rounds > 0 && (!rounds || !mt_dev)))
    return fail(ctx, PVT_EINVAL, "bad batch (%d rounds)", n_rounds);
  ctx->rs.active = false;
  if (n_rounds == 0) return PVT_OK;
  std::vector<pvt_round> rr(rounds, rounds + n_rounds);   // (mt_state: the device rows, so
  for (int i = 0; i < n_rounds; i++) rr[i].mt_state = mt_dev + (size_t)i * 625;   // checks pass)
  return place_resident(ctx, rr.data(), n_rounds, nullptr, mt_dev);
}

// ---------------------------------------------------------------- anchor resolution (a3)
extern "C" int pvt_anchor(pvt_ctx* ctx, const pvt_anchor_args* a) {
  if (!ctx || !a) return PVT_EINVAL;
  if (a->n_items < 0 || a->n_hosts < 0 || a->n_pred < 0 || a->n_inst < 0)
    return fail(ctx, PVT_EINVAL, "negative size in pvt_anchor_args");
  if (a->n_items == 0) return PVT_OK;
  if (!a->off || !a->mode_host || !a->anchor_zone || (a->n_pred > 0 && (!a->list || !a->zone)) ||
      (a->inst_host == nullptr) != (a->n_inst == 0) || (a->item == nullptr) != (a->n_rows == 0))
    return fail(ctx, PVT_EINVAL, "null pointer in pvt_anchor_args");
  (void)hipSetDevice(ctx->device);
  ENSURE(ctx->anc_scr, 16 + sizeof(int32_t) * (size_t)a->n_items);
  int32_t* bad = P<int32_t>(ctx->anc_scr);   // [0] bad items, [1] deferred count, [4..] list
  HIPCHK(hipMemsetAsync(bad, 0, 16, ctx->stream));
  AnchorArgs k{a->n_items, a->n_hosts, a->n_pred, a->n_inst, a->n_rows, a->off, a->item,
               a->list, a->inst_host, a->zone, a->mode_host, a->anchor_zone, bad, bad + 4, bad + 1};
  {
    Scope sc(ctx, PVT_K_OTHER, 0, 4.0 * (double)a->n_pred);
    launch_anchor(k, ctx->stream);
  }
  HIPCHK(hipGetLastError());
  int32_t nbad = 0;
  HIPCHK(hipMemcpyAsync(&nbad, bad, sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  if (nbad) return fail(ctx, PVT_EINVAL, "%d anchor item(s) with invalid offsets or indices", nbad);
  return PVT_OK;
}

// ---------------------------------------------------------------- meter aggregates (f4)
extern "C" int pvt_meter(pvt_ctx* ctx, const pvt_meter_log* m) {
  if (!ctx || !m) return PVT_EINVAL;
  if (m->n_scen < 0 || m->reserved != 0 || m->n_host_rows < 0 || m->n_iv < 0 ||
      m->n_routes < 0 || m->n_pkts < 0 || m->n_tr < 0)
    return fail(ctx, PVT_EINVAL, "bad size in pvt_meter_log");
  if (m->n_scen == 0) return PVT_OK;
  if (!m->host_off || !m->iv_off || !m->route_off || !m->pkt_off || !m->tr_off ||
      !m->instance_hours || !m->egress_cost || !m->congestion_delay ||
      (m->n_iv && (!m->iv_start || !m->iv_end)) || (m->n_routes && !m->route_cost) ||
      (m->n_tr && (!m->tr_start || !m->tr_end || !m->tr_size)))
    return fail(ctx, PVT_EINVAL, "null pointer in pvt_meter_log");
  (void)hipSetDevice(ctx->device);
  ENSURE(ctx->anc_scr, 16);
  int32_t* bad = P<int32_t>(ctx->anc_scr);
  HIPCHK(hipMemsetAsync(bad, 0, sizeof(int32_t), ctx->stream));
  MeterArgs k{m->n_scen, m->n_host_rows, m->n_iv, m->n_routes, m->n_pkts, m->n_tr,
              m->host_off, m->iv_off, m->route_off, m->pkt_off, m->tr_off,
              m->iv_start, m->iv_end, m->route_cost, m->tr_start, m->tr_end, m->tr_size,
              m->instance_hours, m->egress_cost, m->congestion_delay, bad};
  {
    Scope sc(ctx, PVT_K_OTHER, 0, 16.0 * (double)m->n_iv + 24.0 * (double)m->n_tr);
    launch_meter(k, ctx->stream);
  }
  HIPCHK(hipGetLastError());
  int32_t nbad = 0;
  HIPCHK(hipMemcpyAsync(&nbad, bad, sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  if (nbad) return fail(ctx, PVT_EINVAL, "%d scenario(s) with out-of-range meter offsets", nbad);
  return PVT_OK;
}

extern "C" int pvt_set_resident(pvt_ctx* ctx, int32_t max_hosts) {
  if (!ctx || max_hosts < 0) return PVT_EINVAL;
  ctx->resident_max = max_hosts;
  return PVT_OK;
}

// The windowed / epoch / opportunistic engines on a checked round of device arrays (pvt_place
// without the resident case); synchronises before returning.
static int place_windowed(pvt_ctx* ctx, const pvt_round* r) {
  int rc;
  if (r->mode == PVT_OPP) {
    ctx->rs.active = false;
    ctx->windows = ctx->refills = 0;
    HIPCHK(hipSetDevice(ctx->device));
    if (r->n_tasks == 0) return PVT_OK;
    HIPCHK(hipMemsetAsync(r->placement, 0xff, sizeof(int32_t) * r->n_tasks, ctx->stream));
    launch_iota(r->order, r->n_tasks, ctx->stream);
    return opp_round(ctx, r);
  }
  ctx->rs.sharded = false;
  if ((rc = round_begin(ctx, r, 0, r->n_hosts, 1))) return rc;
  ctx->n_epochs = ctx->n_segs = ctx->n_rejected = 0;
  ctx->n_zchains = ctx->n_gchains = ctx->n_longest = 0;
  if ((rc = epoch_groups(ctx))) return rc;
  rc = ctx->rs.egs.empty() ? place_pipelined(ctx) : place_epochs(ctx);
  ctx->rs.active = false;
  if (rc) {
    (void)hipStreamSynchronize(ctx->side);
    return rc;
  }
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return PVT_OK;
}

extern "C" int pvt_place(pvt_ctx* ctx, const pvt_round* r) {
  if (!ctx) return PVT_EINVAL;
  int rc = check_round(ctx, r);
  if (rc) return rc;
  if (r->n_tasks > 0 && resident_fits(r, ctx->resident_max)) {
    ctx->rs.active = false;
    return place_resident(ctx, r, 1);
  }
  return place_windowed(ctx, r);
}

// ---------------------------------------------------------------- drop-in rounds, host memory
static int ensure_pinned(pvt_ctx* ctx, size_t bytes) {
  if (ctx->hst_cap >= bytes) return PVT_OK;
  const size_t want = std::max({bytes, ctx->hst_cap * 3 / 2, (size_t)1 << 16});
  if (ctx->hst) (void)hipHostFree(ctx->hst);
  ctx->hst = nullptr;
  ctx->hst_map = nullptr;
  ctx->hst_cap = 0;
  if (hipHostMalloc(&ctx->hst, want) != hipSuccess) {
    ctx->hst = nullptr;
    return fail(ctx, PVT_ENOMEM, "hipHostMalloc(%zu) failed", want);
  }
  if (hipHostGetDevicePointer(&ctx->hst_map, ctx->hst, 0) != hipSuccess) {
    (void)hipHostFree(ctx->hst);
    ctx->hst = ctx->hst_map = nullptr;
    return fail(ctx, PVT_EHIP, "hipHostGetDevicePointer of the staging buffer failed");
  }
  ctx->hst_cap = want;
  return PVT_OK;
}

// One host-memory round's place in the staging buffer (pvt_place_host, pvt_place_host_batch):
// the out region (copied back: avail, placement, order, MT states, grouping status) of every
// round of a call comes first, so the results return with ONE copy.
struct HostSlot {
  size_t av = 0, pl = 0, orr = 0, mt = 0, cmt = 0, st = 0;
  size_t zone = 0, tb = 0, dc = 0, cost = 0, bw = 0, dem = 0, tg = 0, ga = 0, rt = 0;
  size_t ti = 0, off = 0, ph = 0, ia = 0, sz = 0, zs = 0, mh = 0, az = 0, ab = 0, desc = 0;
  size_t out_lo = 0, out_hi = 0, in_lo = 0, in_hi = 0;   // its byte ranges (fused host batch)
  const double* zt = nullptr;         // device zone tables (cost, then bw) when cached, else NULL
  int C = 0, S = 0, G = 0, GR = 0;
  int64_t NP = 0;
  bool resident = false, dev_mt = false;
  pvt_round hr{};                     // the round as checked (grouped fields stand in with items)
  pvt_round d{};                      // the device round (arrays in the staging buffer)
};

// Validation of a host round and its optional fused-grouping items (pvt_place_host's contract).
static int check_host_round(pvt_ctx* ctx, const pvt_round* r, pvt_ca_items* it, HostSlot& s) {
  const bool ca = r->mode == PVT_CA_FF || r->mode == PVT_CA_BF;
  const int T = r->n_tasks, Z = r->n_zones;
  if (it) {
    if (!ca) return fail(ctx, PVT_EINVAL, "pvt_ca_items need a cost_aware round");
    if (it->reserved != 0 || it->n_items < 0 || it->n_apps < 0 || it->n_pred < 0 || it->n_storage < 0)
      return fail(ctx, PVT_EINVAL, "bad sizes in pvt_ca_items");
    if (r->task_group || r->group_anchor || r->rt_bw)
      return fail(ctx, PVT_EINVAL, "pvt_ca_items replace task_group / group_anchor (realtime_bw "
                  "rows are per group: use pvt_anchor + pvt_place)");
    if (!it->status || (T > 0 && (!it->task_item || !it->pred_off || (it->n_pred && !it->pred_host) ||
                                  (it->n_items && !it->item_app) || !it->storage_zone ||
                                  !it->zone_storage || !it->mt_state)))
      return fail(ctx, PVT_EINVAL, "null pointer in pvt_ca_items");
    it->status[0] = it->status[1] = 0;
    if (T > GRP_MAX_TASKS || it->n_storage + it->n_apps > GRP_MAX_KEYS || it->n_storage < 1)
      return fail(ctx, PVT_EUNSUPPORTED, "fused grouping limits: T=%d (max %d), %d storages + %d "
                  "applications (max %d, at least one storage)", T, GRP_MAX_TASKS, it->n_storage,
                  it->n_apps, GRP_MAX_KEYS);
    if (Z < 1 || Z > ZMAX) return fail(ctx, PVT_EINVAL, "bad sizes H=%d T=%d Z=%d", r->n_hosts, T, Z);
    for (int k = 0; k < it->n_storage; k++)
      if (it->storage_zone[k] < 0 || it->storage_zone[k] >= Z)
        return fail(ctx, PVT_EINVAL, "storage %d: zone %d outside [0, %d)", k, it->storage_zone[k], Z);
    for (int z = 0; z < Z; z++)
      if (it->zone_storage[z] < -1 || it->zone_storage[z] >= it->n_storage)
        return fail(ctx, PVT_EINVAL, "zone %d: storage %d outside [-1, %d)", z, it->zone_storage[z], it->n_storage);
    for (int c = 0; c <= it->n_items && T > 0; c++)   // (the anchor kernels check each range too)
      if (it->pred_off[c] < 0 || it->pred_off[c] > it->n_pred || (c && it->pred_off[c] < it->pred_off[c - 1]))
        return fail(ctx, PVT_EINVAL, "pred_off[%d] = %lld out of order or range", c, (long long)it->pred_off[c]);
  }
  s.hr = *r;
  static const int32_t one = 0;
  if (it) { s.hr.task_group = &one; s.hr.group_anchor = &one; s.hr.n_groups = 1; }
  int rc = check_round(ctx, &s.hr);
  if (rc) return rc;
  if (ca && T > 0)   // host arrays: the zone-table contract of include/pivot_place.h (cost, bw)
    for (int a = 0; a < Z; a++)
      for (int z = 0; z < Z; z++) {
        const double c = r->cost[a * Z + z] + r->cost[z * Z + a], b = r->bw[a * Z + z] + r->bw[z * Z + a];
        if (!(c >= 0.0) || !(b > 0.0))
          return fail(ctx, PVT_EINVAL, "zones (%d, %d): cost sum %g, bw sum %g (the engine needs "
                      "cost sums >= 0 and bw sums > 0)", a, z, c, b);
      }
  s.resident = T > 0 && resident_fits(&s.hr, ctx->resident_max);
  s.C = it ? it->n_items : 0;
  s.S = it ? it->n_storage : 0;
  s.NP = it ? it->n_pred : 0;
  s.G = it ? T : (r->task_group ? r->n_groups : 0);
  s.GR = r->rt_bw ? std::max(r->task_group ? r->n_groups : 1, 1) : 0;
  s.dev_mt = r->mt_state && s.resident;
  return PVT_OK;
}

// The device copy of a host round's zone tables, when they equal the cached ones (s.zt); the
// cache takes the tables of the first cost_aware round of a call that misses it (one small
// copy on the stream; every host-array call ends with a synchronisation, so no kernel of an
// earlier call still reads the old tables).
static int zone_cache(pvt_ctx* ctx, const pvt_round* r, HostSlot& s) {
  s.zt = nullptr;
  if (!r->cost || !r->bw || r->n_tasks == 0) return PVT_OK;
  const int Z = r->n_zones;
  const size_t zz = (size_t)Z * Z;
  auto same = [&]() {
    return ctx->zt_Z == Z && ctx->zt_host.size() == 2 * zz &&
           std::memcmp(ctx->zt_host.data(), r->cost, 8 * zz) == 0 &&
           std::memcmp(ctx->zt_host.data() + zz, r->bw, 8 * zz) == 0;
  };
  if (!same()) {
    ctx->zt_host.resize(2 * zz);
    std::memcpy(ctx->zt_host.data(), r->cost, 8 * zz);
    std::memcpy(ctx->zt_host.data() + zz, r->bw, 8 * zz);
    ctx->zt_Z = Z;
    ENSURE(ctx->zt_dev, 16 * zz);
    HIPCHK(hipMemcpyAsync(ctx->zt_dev.p, ctx->zt_host.data(), 16 * zz, hipMemcpyHostToDevice, ctx->stream));
  }
  s.zt = P<double>(ctx->zt_dev);
  return PVT_OK;
}

struct StageLayout {
  size_t o = 0;
  size_t take(size_t bytes) { const size_t at = o; o = (o + bytes + 255) / 256 * 256; return at; }
};

static void plan_out(StageLayout& L, HostSlot& s, const pvt_round* r, const pvt_ca_items* it) {
  const int H = r->n_hosts, T = r->n_tasks;
  s.out_lo = L.o;
  s.av = L.take(32 * (size_t)H);
  s.pl = L.take(4 * (size_t)T);
  s.orr = L.take(4 * (size_t)T);
  s.mt = r->mt_state ? L.take(4 * 625) : 0;
  s.cmt = it ? L.take(4 * 625) : 0;
  s.st = it ? L.take(16) : 0;
  s.out_hi = L.o;
}

static void plan_in(StageLayout& L, HostSlot& s, const pvt_round* r, const pvt_ca_items* it) {
  const int H = r->n_hosts, T = r->n_tasks, Z = r->n_zones;
  s.in_lo = L.o;
  s.zone = L.take(4 * (size_t)H);
  s.tb = r->tiebreak ? L.take(4 * (size_t)H) : 0;
  s.dc = r->decay ? L.take(4 * (size_t)H) : 0;
  s.cost = s.zt ? 0 : L.take(8 * (size_t)Z * Z);
  s.bw = s.zt ? 0 : L.take(8 * (size_t)Z * Z);
  s.dem = L.take(32 * (size_t)T);
  s.tg = (it || r->task_group) ? L.take(4 * (size_t)T) : 0;
  s.ga = (it || r->task_group) ? L.take(4 * (size_t)std::max(s.G, 1)) : 0;
  s.rt = s.GR ? L.take(8 * (size_t)s.GR * H) : 0;
  if (it) {
    s.ti = L.take(4 * (size_t)T);
    s.off = L.take(8 * (size_t)(s.C + 1));
    s.ph = L.take(4 * (size_t)std::max<int64_t>(s.NP, 1));
    s.ia = L.take(4 * (size_t)std::max(s.C, 1));
    s.sz = L.take(4 * (size_t)s.S);
    s.zs = L.take(4 * (size_t)Z);
    s.mh = L.take(4 * (size_t)std::max(s.C, 1));
    s.az = L.take(4 * (size_t)std::max(s.C, 1));
    s.ab = L.take(16 + 4 * (size_t)std::max(s.C, 1));
  }
  s.in_hi = L.o;
}

// The round's inputs into the pinned buffer and its device descriptor (arrays in the device
// copy of the buffer; a windowed opportunistic round's MT state stays a host pointer: opp_round
// moves it itself).
static void stage_round(char* hb, char* db, HostSlot& s, const pvt_round* r, const pvt_ca_items* it) {
  const int H = r->n_hosts, T = r->n_tasks, Z = r->n_zones;
  auto put = [&](size_t at, const void* src, size_t bytes) { if (bytes) std::memcpy(hb + at, src, bytes); };
  put(s.av, r->avail, 32 * (size_t)H);
  if (r->mt_state) put(s.mt, r->mt_state, 4 * 625);
  if (it) { put(s.cmt, it->mt_state, 4 * 625); std::memset(hb + s.st, 0, 16); }
  put(s.zone, r->zone, 4 * (size_t)H);
  if (r->tiebreak) put(s.tb, r->tiebreak, 4 * (size_t)H);
  if (r->decay) put(s.dc, r->decay, 4 * (size_t)H);
  if (!s.zt) {
    put(s.cost, r->cost, r->cost ? 8 * (size_t)Z * Z : 0);
    put(s.bw, r->bw, r->bw ? 8 * (size_t)Z * Z : 0);
  }
  put(s.dem, r->dem, 32 * (size_t)T);
  if (r->task_group) { put(s.tg, r->task_group, 4 * (size_t)T); put(s.ga, r->group_anchor, 4 * (size_t)s.G); }
  if (s.GR) put(s.rt, r->rt_bw, 8 * (size_t)s.GR * H);
  if (it) {
    put(s.ti, it->task_item, 4 * (size_t)T);
    put(s.off, it->pred_off, 8 * (size_t)(s.C + 1));
    put(s.ph, it->pred_host, 4 * (size_t)s.NP);
    put(s.ia, it->item_app, 4 * (size_t)s.C);
    put(s.sz, it->storage_zone, 4 * (size_t)s.S);
    put(s.zs, it->zone_storage, 4 * (size_t)Z);
    std::memset(hb + s.ab, 0, 16);
  }
  pvt_round& d = s.d;
  d = s.hr;
  d.avail = reinterpret_cast<double*>(db + s.av);
  d.zone = reinterpret_cast<const int32_t*>(db + s.zone);
  d.tiebreak = r->tiebreak ? reinterpret_cast<const uint32_t*>(db + s.tb) : nullptr;
  d.decay = r->decay ? reinterpret_cast<const int32_t*>(db + s.dc) : nullptr;
  d.cost = s.zt ? s.zt : r->cost ? reinterpret_cast<const double*>(db + s.cost) : nullptr;
  d.bw = s.zt ? s.zt + (size_t)Z * Z : r->bw ? reinterpret_cast<const double*>(db + s.bw) : nullptr;
  d.dem = reinterpret_cast<const double*>(db + s.dem);
  d.task_group = s.tg ? reinterpret_cast<const int32_t*>(db + s.tg) : nullptr;
  d.group_anchor = s.ga ? reinterpret_cast<const int32_t*>(db + s.ga) : nullptr;
  d.rt_bw = s.GR ? reinterpret_cast<const double*>(db + s.rt) : nullptr;
  d.placement = reinterpret_cast<int32_t*>(db + s.pl);
  d.order = reinterpret_cast<int32_t*>(db + s.orr);
  d.mt_state = s.dev_mt ? reinterpret_cast<uint32_t*>(db + s.mt) : r->mt_state;
  std::memcpy(hb + s.desc, &d, sizeof(pvt_round));
}

// The fused cost_aware grouping of an items round on the device (anchors, groups, draws); a
// resident round's descriptor receives its group count.
static void items_args(char* db, const HostSlot& s, const pvt_ca_items* it, AnchorArgs* ka,
                       CaGroupArgs* ga) {
  const int T = s.hr.n_tasks, H = s.hr.n_hosts, Z = s.hr.n_zones;
  int32_t* ab = reinterpret_cast<int32_t*>(db + s.ab);
  *ka = AnchorArgs{s.C, H, s.NP, 0, 0, reinterpret_cast<const int64_t*>(db + s.off), nullptr,
                   reinterpret_cast<const int32_t*>(db + s.ph), nullptr, s.d.zone,
                   reinterpret_cast<int32_t*>(db + s.mh), reinterpret_cast<int32_t*>(db + s.az), ab,
                   ab + 4, ab + 1};
  *ga = CaGroupArgs{T, s.C, Z, s.S, it->n_apps, reinterpret_cast<const int32_t*>(db + s.ti),
                    reinterpret_cast<const int32_t*>(db + s.az), reinterpret_cast<const int32_t*>(db + s.ia),
                    reinterpret_cast<const int32_t*>(db + s.sz), reinterpret_cast<const int32_t*>(db + s.zs),
                    reinterpret_cast<uint32_t*>(db + s.cmt), reinterpret_cast<int32_t*>(db + s.tg),
                    reinterpret_cast<int32_t*>(db + s.ga), reinterpret_cast<int32_t*>(db + s.st),
                    s.resident ? &reinterpret_cast<pvt_round*>(db + s.desc)->n_groups : nullptr};
}

static int launch_items(pvt_ctx* ctx, char* db, const HostSlot& s, const pvt_ca_items* it, hipStream_t st) {
  AnchorArgs k;
  CaGroupArgs g;
  items_args(db, s, it, &k, &g);
  {
    Scope sc(ctx, PVT_K_OTHER, 0, 4.0 * (double)s.NP);
    if (s.C > 0) launch_anchor(k, st);
    launch_ca_groups(g, st);
  }
  HIPCHK(hipGetLastError());
  return PVT_OK;
}

static int group_error(pvt_ctx* ctx, const char* hb, const HostSlot& s, pvt_ca_items* it) {
  const int32_t* hs = reinterpret_cast<const int32_t*>(hb + s.st);
  const int e = hs[1];
  it->status[0] = hs[0];
  it->status[1] = e;
  if (!e) return PVT_OK;
  return fail(ctx, PVT_EINVAL, "%s", e == 1 ? "a mode predecessor placement is not a host of the cluster" :
              e == 2 ? "an anchor zone has no storage (get_storage_by_locality -> None)" :
              "malformed anchor item lists");
}

static void return_round(const char* hb, const HostSlot& s, pvt_round* r, pvt_ca_items* it) {
  const int H = r->n_hosts, T = r->n_tasks;
  std::memcpy(r->avail, hb + s.av, 32 * (size_t)H);
  std::memcpy(r->placement, hb + s.pl, 4 * (size_t)T);
  std::memcpy(r->order, hb + s.orr, 4 * (size_t)T);
  if (s.dev_mt) std::memcpy(r->mt_state, hb + s.mt, 4 * 625);
  if (it) std::memcpy(it->mt_state, hb + s.cmt, 4 * 625);
}

// The staging buffer to the device and the results back as copy kernels over its mapped pages:
// a hipMemcpyAsync from or to pinned memory goes through the copy engine, and the next kernel
// on the stream started ~20 us after the copy was queued (launch_upload).
static void stage_up(pvt_ctx* ctx, size_t bytes, hipStream_t st) {
  launch_upload(ctx->hst_map, ctx->hdev.p, bytes, st);
}
static void stage_down(pvt_ctx* ctx, size_t bytes, hipStream_t st) {
  launch_upload(ctx->hdev.p, ctx->hst_map, bytes, st);   // (the same copy kernel, device -> mapped)
}

extern "C" int pvt_place_host(pvt_ctx* ctx, pvt_round* r, pvt_ca_items* it) {
  if (!ctx || !r) return PVT_EINVAL;
  HostSlot s;
  int rc = check_host_round(ctx, r, it, s);
  if (rc) return rc;
  ctx->rs.active = false;
  if (r->n_tasks == 0) return PVT_OK;
  HIPCHK(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  if ((rc = zone_cache(ctx, r, s))) return rc;
  StageLayout L;
  plan_out(L, s, r, it);
  const size_t n_out = L.o;
  plan_in(L, s, r, it);
  s.desc = L.take(sizeof(pvt_round));
  if ((rc = ensure_pinned(ctx, L.o))) return rc;
  ENSURE(ctx->hdev, L.o);
  char* hb = static_cast<char*>(ctx->hst);
  char* db = static_cast<char*>(ctx->hdev.p);
  stage_round(hb, db, s, r, it);
  stage_up(ctx, L.o, st);
  HIPCHK(hipGetLastError());
  if (it && (rc = launch_items(ctx, db, s, it, st))) return rc;
  if (s.resident) {
    if ((rc = place_resident(ctx, &s.d, 1, db + s.desc, s.dev_mt ? reinterpret_cast<uint32_t*>(db + s.mt) : nullptr)))
      return rc;
  } else {
    if (it) {                         // the windowed engine plans groups on the host
      launch_upload(db + s.st, static_cast<char*>(ctx->hst_map) + s.st, 16, st);
      HIPCHK(hipStreamSynchronize(st));
      if ((rc = group_error(ctx, hb, s, it))) return rc;
      s.d.n_groups = std::max(reinterpret_cast<const int32_t*>(hb + s.st)[0], 1);
    }
    if ((rc = place_windowed(ctx, &s.d))) return rc;
  }
  stage_down(ctx, n_out, st);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(st));
  if (it && (rc = group_error(ctx, hb, s, it))) return rc;
  return_round(hb, s, r, it);
  return PVT_OK;
}

extern "C" int pvt_restore_hosts(pvt_ctx* ctx, double* avail, const double* avail0, int32_t n_hosts,
                                 const int32_t* hosts, int32_t n) {
  if (!ctx || n < 0 || n_hosts < 0 || (n > 0 && (!avail || !avail0 || !hosts))) return PVT_EINVAL;
  HIPCHK(hipSetDevice(ctx->device));
  launch_restore_hosts(avail, avail0, n_hosts, hosts, n, ctx->stream);
  HIPCHK(hipGetLastError());
  return PVT_OK;
}

// The staged host batch in ONE launch (resident_fused_kernel, pvt_batch.hip): every round's
// workgroup copies its ranges of the mapped stage to the device copy, runs its grouping (items)
// and its placement, and copies its results back; one synchronisation. PVT_FUSED=0: the staged
// upload / anchor / grouping / placement / download launches instead (A/B).
static int place_host_fused(pvt_ctx* ctx, pvt_round* rounds, pvt_ca_items* const* items,
                            int32_t n_rounds, int32_t* rcs, std::vector<HostSlot>& s,
                            const std::vector<int>& live, const std::vector<int>& withit,
                            size_t o_fr, size_t o_ka, size_t o_kg, bool mixed, int mode0, int maxH,
                            int maxT, int maxZ) {
  hipStream_t st = ctx->stream;
  char* hb = static_cast<char*>(ctx->hst);
  char* db = static_cast<char*>(ctx->hdev.p);
  FusedRound* fr = reinterpret_cast<FusedRound*>(hb + o_fr);
  for (size_t k = 0; k < live.size(); k++) {
    const HostSlot& h = s[live[k]];
    fr[k] = FusedRound{(int64_t)h.out_lo, (int64_t)h.out_hi, (int64_t)h.in_lo, (int64_t)h.in_hi,
                       (int64_t)h.desc, -1, 0};
  }
  for (size_t k = 0; k < withit.size(); k++)
    for (size_t j = 0; j < live.size(); j++)
      if (live[j] == withit[k]) fr[j].items = (int32_t)k;
  int waves = 4, hpl = 1;
  resident_shape(maxH, &waves, &hpl);
  int tpad = 64;
  while (tpad < maxT) tpad <<= 1;
  double cand = 0.0, bytes = 0.0;
  for (int i : live) {
    const double c = (double)rounds[i].n_tasks * rounds[i].n_hosts;
    cand += c;
    bytes += c * bytes_per_candidate(rounds[i].mode);
  }
  const int rwalk = ctx->rwalk && maxH <= RW_MAXH ? ctx->rwalk : 0;
  FusedArgs F{static_cast<const char*>(ctx->hst_map), db, (int64_t)o_fr, (int64_t)o_ka,
              (int64_t)o_kg, ResidentArgs{nullptr, nullptr, maxZ, tpad, ctx->stamps, rwalk}};
  size_t lds = resident_lds_bytes(maxZ, tpad, rwalk != 0);
  if (!withit.empty()) lds = std::max(lds, fused_pre_lds_bytes());
  {
    Scope sc(ctx, PVT_K_SCORE, cand, bytes, nullptr, "resident_fused_kernel");
    launch_fused(mixed ? RES_MIXED : mode0, hpl, (int)live.size(), lds, F, st);
  }
  HIPCHK(hipGetLastError());
  ctx->windows = (int64_t)live.size();
  ctx->refills = 0;
  HIPCHK(hipStreamSynchronize(st));
  for (int i : live) {
    pvt_ca_items* it = items ? items[i] : nullptr;
    if (it && (rcs[i] = group_error(ctx, hb, s[i], it))) continue;
    return_round(hb, s[i], &rounds[i], it);
  }
  (void)n_rounds;
  return PVT_OK;
}

extern "C" int pvt_place_host_batch(pvt_ctx* ctx, pvt_round* rounds, pvt_ca_items* const* items,
                                    int32_t n_rounds, int32_t* rcs) {
  if (!ctx) return PVT_EINVAL;
  if (n_rounds < 0 || (n_rounds > 0 && (!rounds || !rcs)))
    return fail(ctx, PVT_EINVAL, "bad host batch (%d rounds)", n_rounds);
  ctx->rs.active = false;
  if (n_rounds == 0) return PVT_OK;
  std::vector<HostSlot> s(n_rounds);
  int rc;
  // mode0: the first round with tasks (an empty round launches nothing and mixes no modes)
  int maxH = 1, maxT = 1, maxZ = 1, mode0 = -1;
  bool mixed = false;
  for (int i = 0; i < n_rounds; i++) {
    pvt_ca_items* it = items ? items[i] : nullptr;
    rcs[i] = PVT_OK;
    if ((rc = check_host_round(ctx, &rounds[i], it, s[i]))) {
      char msg[64];
      std::snprintf(msg, sizeof(msg), "host batch round %d: ", i);
      ctx->err = msg + ctx->err;
      return rc;
    }
    if (rounds[i].n_tasks > 0 && !s[i].resident)
      return fail(ctx, PVT_EUNSUPPORTED, "host batch round %d: H=%d T=%d exceeds the resident limits "
                  "(%d, %d): place it with pvt_place_host", i, rounds[i].n_hosts, rounds[i].n_tasks,
                  std::min(ctx->resident_max, (int)PVT_RESIDENT_MAX_HOSTS), PVT_RESIDENT_MAX_TASKS);
    if (rounds[i].n_tasks == 0) continue;
    maxH = std::max(maxH, rounds[i].n_hosts);
    maxT = std::max(maxT, rounds[i].n_tasks);
    maxZ = std::max(maxZ, rounds[i].n_zones);
    if (mode0 < 0) mode0 = rounds[i].mode;
    mixed |= rounds[i].mode != mode0;
  }
  HIPCHK(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  // out regions of every round, then the inputs, then the descriptors of the rounds with tasks
  // (contiguous: one resident launch takes them all)
  StageLayout L;
  for (int i = 0; i < n_rounds; i++)
    if (rounds[i].n_tasks > 0) plan_out(L, s[i], &rounds[i], items ? items[i] : nullptr);
  const size_t n_out = L.o;
  {
    bool filled = false;               // (the cache takes the first round's tables at most)
    for (int i = 0; i < n_rounds; i++) {
      if (rounds[i].n_tasks == 0 || !rounds[i].cost) continue;
      const int Z = rounds[i].n_zones;
      const size_t zz = (size_t)Z * Z;
      const bool hit = ctx->zt_Z == Z && ctx->zt_host.size() == 2 * zz &&
                       std::memcmp(ctx->zt_host.data(), rounds[i].cost, 8 * zz) == 0 &&
                       std::memcmp(ctx->zt_host.data() + zz, rounds[i].bw, 8 * zz) == 0;
      if (hit || !filled) {
        if ((rc = zone_cache(ctx, &rounds[i], s[i]))) return rc;
        filled = true;
      }
    }
  }
  for (int i = 0; i < n_rounds; i++)
    if (rounds[i].n_tasks > 0) plan_in(L, s[i], &rounds[i], items ? items[i] : nullptr);
  std::vector<int> live, withit;
  for (int i = 0; i < n_rounds; i++)
    if (rounds[i].n_tasks > 0) {
      live.push_back(i);
      if (items && items[i]) withit.push_back(i);
    }
  if (live.empty()) return PVT_OK;
  // the fused groupings of every cost_aware round: their kernel arguments in the stage, so the
  // anchors and the groups of all of them take three launches
  const int ni = (int)withit.size();
  const size_t o_ka = ni ? L.take(sizeof(AnchorArgs) * ni) : 0;
  const size_t o_kb = ni ? L.take(sizeof(int32_t) * (ni + 1)) : 0;
  const size_t o_kg = ni ? L.take(sizeof(CaGroupArgs) * ni) : 0;
  const size_t o_desc = L.take(sizeof(pvt_round) * live.size());
  for (size_t k = 0; k < live.size(); k++) s[live[k]].desc = o_desc + sizeof(pvt_round) * k;
  const bool fused = ctx->fused != 0;
  const size_t o_fr = fused ? L.take(sizeof(FusedRound) * live.size()) : 0;
  if ((rc = ensure_pinned(ctx, L.o))) return rc;
  ENSURE(ctx->hdev, L.o);
  char* hb = static_cast<char*>(ctx->hst);
  char* db = static_cast<char*>(ctx->hdev.p);
  for (int i : live) stage_round(hb, db, s[i], &rounds[i], items ? items[i] : nullptr);
  int nab = 0;
  for (int k = 0; k < ni; k++) {
    const int i = withit[k];
    AnchorArgs ka;
    CaGroupArgs ga;
    items_args(db, s[i], items[i], &ka, &ga);
    std::memcpy(hb + o_ka + sizeof(AnchorArgs) * k, &ka, sizeof(AnchorArgs));
    std::memcpy(hb + o_kg + sizeof(CaGroupArgs) * k, &ga, sizeof(CaGroupArgs));
    reinterpret_cast<int32_t*>(hb + o_kb)[k] = nab;
    nab += anchor_batch_blocks(s[i].C);
  }
  if (ni) reinterpret_cast<int32_t*>(hb + o_kb)[ni] = nab;
  if (fused) return place_host_fused(ctx, rounds, items, n_rounds, rcs, s, live, withit, o_fr,
                                     o_ka, o_kg, mixed, mode0, maxH, maxT, maxZ);
  stage_up(ctx, L.o, st);
  HIPCHK(hipGetLastError());
  if (ni) {
    double np = 0.0;
    for (int i : withit) np += (double)s[i].NP;
    Scope sc(ctx, PVT_K_OTHER, 0, 4.0 * np);
    launch_anchor_batch(reinterpret_cast<const AnchorArgs*>(db + o_ka),
                        reinterpret_cast<const int32_t*>(db + o_kb), ni, nab, st);
    launch_ca_groups_batch(reinterpret_cast<const CaGroupArgs*>(db + o_kg), ni, st);
  }
  HIPCHK(hipGetLastError());
  // one resident launch for every round (one workgroup each; mixed policies branch per
  // workgroup), the MT states read and written through each descriptor's mt_state
  {
    int waves = mixed ? 4 : ctx->res_waves, hpl = 1;
    resident_shape(maxH, &waves, &hpl);
    int tpad = 64;
    while (tpad < maxT) tpad <<= 1;
    double cand = 0.0, bytes = 0.0;
    for (int i : live) {
      const double c = (double)rounds[i].n_tasks * rounds[i].n_hosts;
      cand += c;
      bytes += c * bytes_per_candidate(rounds[i].mode);
    }
    ResidentArgs ra{db + o_desc, nullptr, maxZ, tpad, ctx->stamps,
                    ctx->rwalk && maxH <= RW_MAXH ? ctx->rwalk : 0};
    Scope sc(ctx, PVT_K_SCORE, cand, bytes, nullptr, "resident_kernel");
    launch_resident(mixed ? RES_MIXED : mode0, waves, hpl, (int)live.size(), ra, st);
  }
  HIPCHK(hipGetLastError());
  ctx->windows = (int64_t)live.size();
  ctx->refills = 0;
  stage_down(ctx, n_out, st);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(st));
  for (int i : live) {
    pvt_ca_items* it = items ? items[i] : nullptr;
    if (it && (rcs[i] = group_error(ctx, hb, s[i], it))) continue;
    return_round(hb, s[i], &rounds[i], it);
  }
  return PVT_OK;
}

// ---------------------------------------------------------------- host-dimension sharding
static int shard_depth(int world) { return std::max(KL, LMAX / std::max(world, 1)); }
static int64_t frontier_pkg_bytes(int nslots) {
  return (int64_t)sizeof(FrontierHdr) + (int64_t)sizeof(FrontierSlot) * nslots;
}

// ---- host-sharded opportunistic rounds (per-rank feasible counts, exchanged;
// the draw and the k-th selection replicated). Each rank counts its super-chunks of a window
// (bitmaps + counts, task-major) into its package; after the all-gather every rank unpacks the
// full tables and runs the same commit walk, so placements, availability and the MT19937 state
// are identical on all ranks and equal to pvt_place()'s.
static constexpr int OPP_SHARD_WINDOW = OPP_WINDOW_DEFAULT;
static constexpr int OPP_SUP_HOSTS = OPP_SUP * OPP_CH;

static size_t opp_pkg_bytes(const RoundState& R, int nt) {
  return (size_t)nt * R.opp_Psq * OPP_SUP * 4 * sizeof(uint64_t) + (size_t)nt * R.opp_Psq * sizeof(int32_t);
}
static size_t opp_table_bytes(const RoundState& R) {   // full bitmaps + counts of one window
  return (((size_t)R.opp_W * R.opp_nq * 4 * sizeof(uint64_t) + (size_t)R.opp_W * R.opp_nsq * sizeof(int32_t)) + 255) / 256 * 256;
}

static int opp_shard_begin(pvt_ctx* ctx, const pvt_round* r, int lo, int hi, int world,
                           int64_t* max_package_bytes) {
  RoundState& R = ctx->rs;
  const int H = r->n_hosts, T = r->n_tasks;
  if (!r->mt_state) return fail(ctx, PVT_EINVAL, "opportunistic needs mt_state");
  R.r = *r;
  R.T = T; R.H = H; R.Z = r->n_zones; R.lo = lo; R.hi = hi; R.world = world;
  R.t0 = 0; R.nt = 0; R.opp = true;
  R.opp_W = OPP_SHARD_WINDOW;
  R.opp_nq = (H + OPP_CH - 1) / OPP_CH;
  R.opp_nsq = (R.opp_nq + OPP_SUP - 1) / OPP_SUP;
  R.opp_Psq = (R.opp_nsq + world - 1) / world;
  if ((lo % OPP_SUP_HOSTS != 0 && lo != H) || (hi != H && hi % OPP_SUP_HOSTS != 0) ||
      hi - lo > R.opp_Psq * OPP_SUP_HOSTS)
    return fail(ctx, PVT_EINVAL, "opportunistic shard [%d, %d) must span whole super-chunks of %d hosts, "
                "at most %d of them (rank r: [r*%d, (r+1)*%d) clamped to H)", lo, hi, OPP_SUP_HOSTS,
                R.opp_Psq, R.opp_Psq * OPP_SUP_HOSTS, R.opp_Psq * OPP_SUP_HOSTS);
  R.opp_sq_lo = lo < hi ? lo / OPP_SUP_HOSTS : 0;    // an empty shard counts nothing
  R.opp_sq_hi = lo < hi ? (hi + OPP_SUP_HOSTS - 1) / OPP_SUP_HOSTS : 0;
  if (max_package_bytes) *max_package_bytes = (int64_t)opp_pkg_bytes(R, R.opp_W);
  HIPCHK(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  if (T > 0) {
    HIPCHK(hipMemsetAsync(r->placement, 0xff, sizeof(int32_t) * T, st));
    launch_iota(r->order, T, st);
    ENSURE(ctx->dem_ord, sizeof(double) * 4 * T);
    launch_gather_tasks(r->dem, r->order, nullptr, nullptr, T, P<double>(ctx->dem_ord), nullptr,
                        nullptr, st);
    ENSURE(ctx->opp, opp_table_bytes(R) + sizeof(uint32_t) * 640);
    uint32_t* mt = reinterpret_cast<uint32_t*>(P<char>(ctx->opp) + opp_table_bytes(R));
    HIPCHK(hipMemcpyAsync(mt, r->mt_state, sizeof(uint32_t) * 625, hipMemcpyHostToDevice, st));
  }
  ENSURE(ctx->oppfault, 16);
  HIPCHK(hipMemsetAsync(ctx->oppfault.p, 0, sizeof(int32_t), st));   // the walks' fault word
  R.active = true;
  return PVT_OK;
}

static int opp_shard_score(pvt_ctx* ctx, void* package, int32_t* n_tasks_out, int64_t* package_bytes) {
  RoundState& R = ctx->rs;
  hipStream_t st = ctx->stream;
  if (R.t0 >= R.T) {                          // done: the MT19937 state back to the caller
    if (R.T > 0) {
      uint32_t* mt = reinterpret_cast<uint32_t*>(P<char>(ctx->opp) + opp_table_bytes(R));
      HIPCHK(hipMemcpyAsync(R.r.mt_state, mt, sizeof(uint32_t) * 625, hipMemcpyDeviceToHost, st));
    }
    HIPCHK(hipMemcpyAsync(ctx->next_host + 3, ctx->oppfault.p, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    R.active = false;
    if (ctx->next_host[3])
      return fail(ctx, PVT_EHIP, "opportunistic walk: inconsistent feasible counts");
    return PVT_OK;
  }
  const int nt = std::min(R.opp_W, R.T - R.t0);
  const int nsr = std::max(0, R.opp_sq_hi - R.opp_sq_lo);
  uint64_t* bm = reinterpret_cast<uint64_t*>(package);
  int32_t* sc = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(package) +
                                           (size_t)nt * R.opp_Psq * OPP_SUP * 4 * sizeof(uint64_t));
  if (nsr > 0) {
    OppCountArgs ca{R.r.avail, P<double>(ctx->dem_ord) + (size_t)R.t0 * 4, R.H, nt, 0, 0,
                    R.opp_nq, R.opp_nsq, nt, bm, sc, R.opp_sq_lo, R.opp_sq_hi,
                    R.opp_Psq * OPP_SUP, R.opp_Psq};
    Scope s(ctx, PVT_K_SCORE, (double)nt * (R.hi - R.lo), (double)nt * (R.hi - R.lo) * 32.0);
    launch_opp_count(ca, st);
  }
  HIPCHK(hipGetLastError());
  R.nt = nt;
  ctx->windows++;
  *n_tasks_out = nt;
  *package_bytes = (int64_t)opp_pkg_bytes(R, nt);
  HIPCHK(hipStreamSynchronize(st));           // the package is complete when this returns
  return PVT_OK;
}

static int opp_shard_commit(pvt_ctx* ctx, const void* packages) {
  RoundState& R = ctx->rs;
  const pvt_round* r = &R.r;
  hipStream_t st = ctx->stream;
  const int nt = R.nt, t0 = R.t0;
  char* base = P<char>(ctx->opp);
  uint64_t* bm = reinterpret_cast<uint64_t*>(base);
  int32_t* sc = reinterpret_cast<int32_t*>(base + (size_t)R.opp_W * R.opp_nq * 4 * sizeof(uint64_t));
  uint32_t* mt = reinterpret_cast<uint32_t*>(base + opp_table_bytes(R));
  OppUnpackArgs ua{reinterpret_cast<const uint8_t*>(packages), (int64_t)opp_pkg_bytes(R, nt),
                   R.world, nt, R.opp_nq, R.opp_nsq, R.opp_Psq, R.opp_W, bm, sc};
  {
    Scope s(ctx, PVT_K_MERGE, 0, 0);
    launch_opp_unpack(ua, st);
  }
  OppCommitArgs oa{r->avail, P<double>(ctx->dem_ord) + (size_t)t0 * 4, bm, sc, R.H, nt, R.opp_nq,
                   R.opp_nsq, R.opp_W, r->placement + t0, mt, ctx->stamps, nullptr, nullptr, 1,
                   P<int32_t>(ctx->oppfault)};
  {
    Scope s(ctx, PVT_K_COMMIT, 0, 0, nullptr, "opp_commit_kernel");
    launch_opp_commit(oa, st);
  }
  HIPCHK(hipGetLastError());
  R.t0 += nt;
  R.nt = 0;
  return PVT_OK;
}

extern "C" int pvt_shard_begin(pvt_ctx* ctx, const pvt_round* r, int32_t host_lo,
                               int32_t host_hi, int32_t world, int64_t* max_package_bytes) {
  if (!ctx || !r) return PVT_EINVAL;
  ctx->rs.active = false;
  if (world < 1 || world > PVT_SHARD_MAX_WORLD)
    return fail(ctx, PVT_EINVAL, "world %d outside [1, %d]", world, PVT_SHARD_MAX_WORLD);
  if (host_lo < 0 || host_hi < host_lo || host_hi > r->n_hosts)
    return fail(ctx, PVT_EINVAL, "bad host range [%d, %d) of %d", host_lo, host_hi, r->n_hosts);
  ctx->rs.opp = false;
  ctx->rs.inflight = ctx->rs.spec = false;
  ctx->rs.nt = 0;
  ctx->rs.pkind = PK_LIST;
  ctx->n_epochs = ctx->n_segs = ctx->n_rejected = 0;
  ctx->n_zchains = ctx->n_gchains = ctx->n_longest = 0;
  if (r->mode == PVT_OPP) {
    int rc = check_round(ctx, r);
    if (rc) return rc;
    ctx->windows = ctx->refills = 0;
    return opp_shard_begin(ctx, r, host_lo, host_hi, world, max_package_bytes);
  }
  RoundState& R = ctx->rs;
  R.sharded = true;
  int rc = round_begin(ctx, r, host_lo, host_hi, world);
  if (rc) return rc;
  // cost_aware best-fit: frontier-walked epochs (the walk's exchange is its window candidates),
  // list windows for what they cannot prove
  if ((rc = epoch_groups(ctx))) return rc;
  R.sh_epochs = !R.egs.empty() && ctx->zwalk && !R.r.rt_bw && R.Z <= ZMAX;
  R.list_until = 0;
  if (R.sh_epochs) {
    ENSURE(ctx->ep_dev, sizeof(int32_t) * EP_WORDS);
    ENSURE(ctx->wres, sizeof(WinRec) * (size_t)EPOCH_MAX);
    ENSURE(ctx->hmin, sizeof(double) * 4 * ZW_MIN_PARTS);
  }
  if (R.sh_epochs || R.ofront || R.keyed) {
    ENSURE(ctx->fwin, sizeof(FrontierSlot) * (size_t)EPOCH_SEGS);
    ENSURE(ctx->hmin, sizeof(double) * 4 * ZW_MIN_PARTS);
  }
  const int PK = shard_depth(world);
  ENSURE(ctx->pkg, sizeof(SegEntry) * (size_t)(PK + 1) * R.Wmax);
  const int64_t lists = (int64_t)sizeof(SegEntry) * (PK + 1) * R.Wmax;
  if (max_package_bytes) *max_package_bytes = std::max(lists, frontier_pkg_bytes(EPOCH_SEGS));
  return PVT_OK;
}

// The walk in flight, waited for: the round continues where it stopped.
static int shard_finish_walk(pvt_ctx* ctx) {
  RoundState& R = ctx->rs;
  if (!R.inflight) return PVT_OK;
  R.inflight = false;
  int adv = 0, rc;
  if ((rc = walk_status(ctx, R.if_t0, R.if_nt, R.if_inh, &adv))) return rc;
  adapt_window(ctx, adv, R.if_nt);
  R.t0 = R.if_t0 + adv;
  R.of_try = R.ofront;            // (place_pipelined: ordered_frontier after every list walk)
  return PVT_OK;
}

// Last task (exclusive) a list window starting at t0 may reach: keyed rounds stop at the group
// end (frozen keys), sharded best-fit epochs at list_until (frontier epochs go on from there).
static int list_end(const RoundState& R, int t0) {
  int ge = group_end(R, t0);
  if (R.sh_epochs) ge = std::min(ge, std::max(R.list_until, t0));
  return ge;
}

// ---- host-sharded frontier walks. A step's package is this rank's window candidates
// (FrontierHdr, then a FrontierSlot per epoch chain or for the one keyed / ordered walk); after
// the all-gather every rank merges them (launch_zwin_merge) into exactly the window the unsharded
// walk builds over all hosts, and runs the same walk, validation and apply on identical inputs.
// Returns with *made = false when the next step is a list window.
static int shard_frontier_score(pvt_ctx* ctx, void* package, int* nt_out, int64_t* bytes_out,
                                bool* made) {
  RoundState& R = ctx->rs;
  const pvt_round* r = &R.r;
  hipStream_t st = ctx->stream;
  *made = false;
  FrontierHdr* hdr = reinterpret_cast<FrontierHdr*>(package);
  FrontierSlot* slots = reinterpret_cast<FrontierSlot*>(hdr + 1);
  if (R.sh_epochs && R.t0 < R.T && R.t0 >= R.list_until) {
    epoch_plan(R, R.t0, R.E);
    const int nch = (int)R.E.segs.size(), nt = R.E.off.back();
    if (nch <= 1) {                 // one chain: list windows (as place_epochs)
      R.list_until = R.t0 + nt;
      return PVT_OK;
    }
    int rc;
    if ((rc = upload_chain_tables(ctx, R.E))) return rc;
    int32_t* dev = P<int32_t>(ctx->ep_dev);
    {
      Scope sc(ctx, PVT_K_OTHER, 0, 0);
      launch_host_min(r->avail, R.H, R.lo, R.hi, &hdr->hmin[0][0], st);
      ZwinArgs za{r->avail, r->zone, R.H, R.Z, R.lo, R.hi, P<double>(ctx->csum),
                  P<int32_t>(ctx->anc_ord) + R.t0, dev + EP_COFF, dev + EP_CMAP, slots};
      launch_zwin_build(za, nch, st);
    }
    ctx->n_epochs++;
    ctx->n_segs += (int)R.E.chain.size();
    R.pkind = PK_EPOCH;
    *nt_out = nt;
    *bytes_out = frontier_pkg_bytes(nch);
    *made = true;
  } else if (R.ofront && R.of_try && R.T - R.t0 >= ORDERED_FRONTIER_MIN) {
    // this rank's first hosts alive for the next tasks' smallest demand, among the first R.ofh
    // hosts of the cluster (ordered_frontier)
    const int n = std::min(R.T - R.t0, R.of_tasks);
    const int hs = std::min(R.ofh, R.H);
    const int he = std::min(R.hi, hs), nloc = std::max(0, he - R.lo);
    const double* dem = P<double>(ctx->dem_ord) + (size_t)R.t0 * 4;
    {
      Scope sc(ctx, PVT_K_OTHER, 0, 0);
      launch_alive_flags(r->avail, R.H, R.lo, he, dem, n, r->mode == PVT_CA_FF ? 1 : 0,
                         P<double>(ctx->hmin), P<uint8_t>(ctx->kflag), st);
      if (nloc > 0) {
        size_t tmp = ctx->ksorttmp.n;
        HIPCHK(hipcub::DeviceSelect::Flagged(P<void>(ctx->ksorttmp), tmp, P<int32_t>(ctx->kiota),
                                             P<uint8_t>(ctx->kflag), P<int32_t>(ctx->kperm),
                                             P<int32_t>(ctx->next) + 2, nloc, st));
      } else {
        HIPCHK(hipMemsetAsync(P<int32_t>(ctx->next) + 2, 0, sizeof(int32_t), st));
      }
      launch_zwin_gather(r->avail, R.H, R.lo, P<int32_t>(ctx->kperm), P<int32_t>(ctx->next) + 2,
                         slots, st);
    }
    R.pkind = PK_ORDERED;
    R.of_n = n;
    R.of_hs = hs;
    *nt_out = n;
    *bytes_out = frontier_pkg_bytes(1);
    *made = true;
  }
  if (*made) {
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(st));   // the package is complete when pvt_shard_score returns
  }
  return PVT_OK;
}

// Keyed first-fit at a group start (round_next_window set kf_pending): this rank's first hosts
// of the group's zero-key prefix (its own sorted range, kperm; length on the device).
static int shard_keyed_score(pvt_ctx* ctx, void* package, int* nt_out, int64_t* bytes_out) {
  RoundState& R = ctx->rs;
  hipStream_t st = ctx->stream;
  FrontierSlot* slots = reinterpret_cast<FrontierSlot*>(reinterpret_cast<FrontierHdr*>(package) + 1);
  {
    Scope sc(ctx, PVT_K_OTHER, 0, 0);
    launch_zwin_gather(R.r.avail, R.H, R.lo, P<int32_t>(ctx->kperm), P<int32_t>(ctx->next) + 2,
                       slots, st);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(st));
  R.pkind = PK_KEYED;
  *nt_out = group_end(R, R.t0) - R.t0;
  *bytes_out = frontier_pkg_bytes(1);
  return PVT_OK;
}

// The exchanged frontier packages: merge, walk, and (epochs) validate + apply; the round goes on
// from the tasks the walk proved. Synchronous.
static int shard_frontier_commit(pvt_ctx* ctx, const void* packages) {
  RoundState& R = ctx->rs;
  const pvt_round* r = &R.r;
  hipStream_t st = ctx->stream;
  const int kind = R.pkind, nt = R.nt, t0 = R.t0;
  const int nslots = kind == PK_EPOCH ? (int)R.E.segs.size() : 1;
  FrontierSlot* win = P<FrontierSlot>(ctx->fwin);
  {
    Scope sc(ctx, PVT_K_MERGE, 0, 0);
    launch_zwin_merge(reinterpret_cast<const uint8_t*>(packages), R.pbytes, R.world, nslots, win,
                      kind == PK_EPOCH ? P<double>(ctx->hmin) : nullptr, st);
  }
  R.nt = 0;
  R.pkind = PK_LIST;
  int rc;
  if (kind == PK_EPOCH) {
    const EpochPlan& E = R.E;
    const int nseg = (int)E.chain.size(), nch = nslots;
    int32_t* dev = P<int32_t>(ctx->ep_dev);
    ENSURE(ctx->cmax, sizeof(double) * 4 * EPOCH_SEGS);
    ZwalkArgs za{r->avail, r->zone, R.H, R.Z, P<double>(ctx->dem_ord) + (size_t)t0 * 4,
                 P<int32_t>(ctx->anc_ord) + t0, R.ord + t0, P<double>(ctx->csum),
                 P<double>(ctx->bsum), dev + EP_COFF, dev + EP_CMAP, dev + EP_STATUS,
                 P<WinRec>(ctx->wres), r->placement, P<double>(ctx->hmin), ctx->stamps,
                 nullptr, 0, 0, 0, nullptr, nullptr, win, dev + EP_CSOFF, dev + EP_CSEG,
                 P<double>(ctx->cmax)};
    {
      Scope sc(ctx, PVT_K_COMMIT, 0, 0, nullptr, "zwalk_kernel");
      launch_zwalk(za, nch, st);
    }
    EpochArgs ea{P<double>(ctx->dem_ord) + (size_t)t0 * 4, P<int32_t>(ctx->anc_ord) + t0,
                 P<double>(ctx->csum), P<double>(ctx->bsum), r->zone, dev + EP_SEG_OFF,
                 dev + EP_SEG_CHAIN, dev + EP_SEG_CSTART, dev + EP_STATUS, P<WinRec>(ctx->wres),
                 r->avail, R.H, R.Z, nt, nseg, dev + EP_BAD, r->rt_bw, P<int32_t>(ctx->grp_ord) + t0,
                 0, P<double>(ctx->cmax), dev + EP_COFF, nch, dev + EP_SAFE};
    {
      Scope sc(ctx, PVT_K_OTHER, 0, 0);
      launch_epoch_validate(ea, st);
      launch_epoch_accept_apply(ea, dev + EP_RES, nch, st, ctx->ep_hdev + EP_STATUS,
                                EP_WORDS - EP_STATUS);   // (readback: mapped)
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(st));
    int need = 0, adv = 0;
    if ((rc = epoch_frontier_verdict(ctx, E, t0, &need, &adv))) return rc;
    // chains the walk could not prove: list windows over the rest of this epoch's tasks
    if (need && adv < nt) R.list_until = t0 + nt;
    R.t0 = t0 + adv;
    return PVT_OK;
  }
  // keyed / ordered: one walk over the merged window, capacities written back
  const bool strict = r->mode == PVT_CA_FF;
  const int n = kind == PK_ORDERED ? R.of_n : nt;
  ENSURE(ctx->wres, sizeof(WinRec) * (size_t)n);
  const double* dem = P<double>(ctx->dem_ord) + (size_t)t0 * 4;
  ZwalkArgs za{r->avail, r->zone, R.H, R.Z, dem, P<int32_t>(ctx->anc_ord) + t0, R.ord + t0,
               nullptr, nullptr, nullptr, nullptr, P<int32_t>(ctx->next), P<WinRec>(ctx->wres),
               r->placement, nullptr, ctx->stamps, nullptr, 0, R.lo, n, r->avail, nullptr, win};
  {
    Scope sc(ctx, PVT_K_COMMIT, 0, 0, nullptr, "zwalk_kernel");
    launch_zwalk_keyed(za, strict, st);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(ctx->next_host, P<int32_t>(ctx->next), sizeof(int32_t) * 2,
                        hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(ctx->next_host + 2, &win->total, sizeof(int32_t), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  const int done = ctx->next_host[0];
  if (done < 0 || done > n) return fail(ctx, PVT_EHIP, "sharded frontier walk returned %d of %d", done, n);
  ctx->n_zchains += done > 0;
  R.t0 = t0 + done;
  if (kind == PK_KEYED) {
    R.kf_pending = false;
    return PVT_OK;
  }
  // ordered: as ordered_frontier -- a short window that stopped the walk doubles the span, an
  // attempt that placed too few tasks hands over to one list window
  const bool short_window = ctx->next_host[2] < ZW_M && R.of_hs < R.H;
  if (done < n && short_window) {
    R.ofh = (int)std::min<int64_t>((int64_t)R.ofh * 2, R.H);
    if (done == 0) return PVT_OK;
  }
  if (done < ORDERED_FRONTIER_MIN) R.of_try = false;
  return PVT_OK;
}

// Pipelined (pvt_set_pipeline, default on): while walk k runs, window k+1 of the same group is
// scored on the side stream -- on the state walk k-1 left -- and its package returned for the
// exchange, which the caller overlaps with walk k; pvt_shard_commit then waits for walk k and
// returns PVT_ESTALE if it stopped early (every rank sees the same walk, so all ranks agree).
extern "C" int pvt_shard_score(pvt_ctx* ctx, void* package, int32_t* n_tasks_out,
                               int64_t* package_bytes) {
  if (!ctx || !package || !n_tasks_out || !package_bytes) return PVT_EINVAL;
  *n_tasks_out = 0;
  *package_bytes = 0;
  RoundState& R = ctx->rs;
  if (!R.active || R.world < 1) return fail(ctx, PVT_EINVAL, "no sharded round in progress");
  if (R.nt != 0) return fail(ctx, PVT_EINVAL, "pvt_shard_score called twice without pvt_shard_commit");
  if (R.opp) return opp_shard_score(ctx, package, n_tasks_out, package_bytes);
  const int PK = shard_depth(R.world);
  int nt = 0, rc, lb = 0;
  hipStream_t st = ctx->stream;
  R.spec = false;
  if (R.inflight) {
    const int t1 = R.if_t0 + R.if_nt, ge = list_end(R, R.if_t0);
    // (ordered rounds: no speculative window; the frontier walk is tried after each)
    if (ctx->pipeline && t1 < ge && !R.ofront) {   // speculative: the window after the walk in flight
      nt = std::min(R.W, ge - t1);
      lb = 1 - R.if_lb;
      st = ctx->side;
      HIPCHK(hipStreamWaitEvent(st, ctx->ev_walk, 0));
      if ((rc = window_lists(ctx, t1, nt, lb, st))) return rc;
      R.spec = true;
      R.pt0 = t1;
    } else if ((rc = shard_finish_walk(ctx))) {
      return rc;
    }
  }
  if (!R.spec) flush_touched(ctx);   // (no band score in flight)
  if (!R.spec) {
    bool made = false;
    int64_t fb = 0;
    if ((rc = shard_frontier_score(ctx, package, &nt, &fb, &made))) return rc;
    if (!made) {
      if ((rc = round_next_window(ctx, &nt))) return rc;
      if (nt > 0 && R.kf_pending) {
        if ((rc = shard_keyed_score(ctx, package, &nt, &fb))) return rc;
        made = true;
      }
    }
    if (made) {
      R.nt = nt;
      R.pt0 = R.t0;
      R.pbytes = fb;
      *n_tasks_out = nt;
      *package_bytes = fb;
      return PVT_OK;
    }
    if (nt == 0) {
      R.active = false;
      HIPCHK(hipStreamSynchronize(ctx->stream));
      return PVT_OK;
    }
    if (R.sh_epochs) nt = std::min(nt, list_end(R, R.t0) - R.t0);
    if ((rc = window_lists(ctx, R.t0, nt, lb, st))) return rc;
    R.pt0 = R.t0;
  }
  R.pkind = PK_LIST;
  Lists L;
  lists_from(ctx, L, lb);
  PackArgs pa{L, nt, PK, R.ordered ? 1 : 0, reinterpret_cast<SegEntry*>(package)};
  {
    Scope sc(ctx, PVT_K_MERGE, 0, 0, st);
    launch_pack(pa, st);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(st));           // the package is complete when this returns
  R.nt = nt;
  R.plb = lb;
  *n_tasks_out = nt;
  *package_bytes = (int64_t)sizeof(SegEntry) * (PK + 1) * nt;
  return PVT_OK;
}

extern "C" int pvt_shard_commit(pvt_ctx* ctx, const void* packages) {
  if (!ctx || !packages) return PVT_EINVAL;
  RoundState& R = ctx->rs;
  if (!R.active || R.nt == 0) return fail(ctx, PVT_EINVAL, "pvt_shard_commit without a scored window");
  if (R.opp) return opp_shard_commit(ctx, packages);
  if (R.pkind != PK_LIST) return shard_frontier_commit(ctx, packages);
  int rc, n_prev = 0;
  if (R.spec) {                               // wait for the walk the package speculated past
    if ((rc = shard_finish_walk(ctx))) return rc;
    if (R.t0 != R.pt0) {                      // it stopped early: the package is stale
      R.nt = 0;
      R.spec = false;
      return PVT_ESTALE;
    }
    n_prev = ctx->next_host[1];               // its hosts: stale in these lists, so touched
  }
  const int PK = shard_depth(R.world), t0 = R.pt0, nt = R.nt, lb = R.plb;
  flush_touched(ctx);   // the walk before: its package's score pass has completed
  Lists L;
  lists_from(ctx, L, lb);
  MergeArgs ma{reinterpret_cast<const SegEntry*>(packages), nullptr, R.r.avail, R.r.zone,
               P<double>(ctx->dem_ord) + (size_t)t0 * 4, P<int32_t>(ctx->anc_ord) + t0,
               R.ord + t0, R.H, nt, R.world, PK, L, nullptr, ctx->t_merge_bitonic};
  {
    Scope sc(ctx, PVT_K_MERGE, 0, 0, nullptr, merge_kernel_name(ma));
    launch_merge(ma, ctx->stream);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(ctx->ev_walk, ctx->stream));   // releases the next speculative score
  if ((rc = walk_launch(ctx, t0, nt, lb, n_prev))) return rc;
  R.inflight = true;
  R.if_t0 = t0; R.if_nt = nt; R.if_lb = lb; R.if_inh = R.spec;
  R.nt = 0;
  if (!ctx->pipeline) return shard_finish_walk(ctx);
  return PVT_OK;
}
