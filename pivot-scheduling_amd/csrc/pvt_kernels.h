// pvt_kernels.h — device data layout and kernel launch interface of the placement engine.
//
// Layout in HBM (all fp64 math is IEEE, no contraction):
//   hosts   avail[4][H] SoA fp64 (cpus, mem, disk, gpus), zone[H] i32, tiebreak[H] u32
//   tasks   processing order ord[T] i32; dem_ord[T][4] fp64 task-major (one 32-B row per
//           task, so a wave reads a task's demand with one scalar load); anc_ord[T] i32
//   zones   csum[Z][Z] = cost[a][z] + cost[z][a], bsum[Z][Z] = bw[a][z] + bw[z][a]
//   lists   per window task: KL candidates, sorted by (score, tiebreak, host) ascending
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

namespace pvt {

// Timed launches (pvt_set_profiling 2: HIP events around one named kernel). Every launch helper
// starts its kernel through PVT_LAUNCH. When the profiling scope (pvt_capi.hip Scope) has armed a
// pair of events, the first launch binds them to the kernel's own dispatch
// (hipExtLaunchKernelGGL: the events take the dispatch's start and end timestamps), so the timed
// kernel costs the stream no marker packets. A recorded event pair around a launch left ~5 us of
// idle GPU on each side of it (config-5 kernel trace: 7.7 us before the frontier walk, 5.0 after).
// `extra` counts launches past the first while armed (a scope that would time only part of its
// work; the scope then drops the sample).
struct TimedEvents {
  hipEvent_t a = nullptr, b = nullptr;
  bool armed = false;
  int used = 0, extra = 0;
};
extern thread_local TimedEvents g_timed;
#define PVT_LAUNCH(kernel, grid, block, shmem, stream, ...)                                         \
  do {                                                                                             \
    ::pvt::TimedEvents& te_ = ::pvt::g_timed;                                                      \
    if (te_.armed && te_.a) {                                                                      \
      hipExtLaunchKernelGGL(kernel, grid, block, shmem, stream, te_.a, te_.b, 0u, __VA_ARGS__);    \
      te_.a = nullptr;                                                                             \
      te_.used++;                                                                                  \
    } else {                                                                                       \
      if (te_.armed) te_.extra++;                                                                  \
      hipLaunchKernelGGL(kernel, grid, block, shmem, stream, __VA_ARGS__);                         \
    }                                                                                              \
  } while (0)

constexpr int WAVE = 64;
constexpr int KL = 64;           // candidate list length per task (one entry per lane)
constexpr int ZMAX = 32;         // zones supported (locality.yml has 31)
constexpr int TW = 4;            // tasks per wave in the score kernel
constexpr int WPB = 4;           // waves per score-kernel block
constexpr int MAX_WINDOW = 1024; // tasks per window (bounded by the commit kernel's LDS)
constexpr int HASH_BITS = 12;    // commit kernel touched-host hash: 4096 slots
constexpr int MAX_SEG = 16;      // host segments per task at a full window
constexpr int CHAIN_MAX = 2048;  // tasks per epoch chain walk (touched-host hash: 4096 slots)

enum Mode { CA_FF = 0, CA_BF = 1, OPP = 2, VBP_FF = 3, VBP_BF = 4 };

struct SegEntry {    // 16 B: one candidate in a per-segment list
  double s;
  uint32_t tb;
  int32_t id;
};

// One candidate of a merged list: 64 B, so lane j of the commit walk reads entry j with
// four 16-B loads.
struct ListEntry {
  double s;           // score (sort key)
  uint32_t tb;        // tiebreak (host-id rank for vbp best-fit, else 0)
  int32_t id;         // host index
  int32_t zone;
  int32_t pad;
  double a[4];        // snapshot availability of the host
  double pad2;
};
// Per window task (64 B, read by lanes 0-15 of the commit walk with one vector load).
struct TaskRec {
  double d[4];
  int32_t cnt;        // valid entries (<= LMAX)
  int32_t complete;   // 1 if every snapshot-feasible host is in the list
  int32_t anc;
  int32_t ord;        // caller index of the task (where its placement is written)
  double bs;          // bound: every snapshot-feasible host NOT in the list has
  uint32_t btb;       //   (score, tiebreak, host) >= (bs, btb, bid)
  int32_t bid;
};
// Merged (final) candidate lists of one window: the exact top-cnt hosts of each task, up to
// LMAX of them (the union of the segment lists is exact below the smallest last entry of an
// incomplete segment list).
constexpr int LMAX = 1024;
struct Lists {
  ListEntry* e;       // [W][LMAX]
  int32_t* ids;       // [W][LMAX] host index of each entry (compact copy for deep searches)
  TaskRec* t;         // [W]
};

struct ScoreArgs {
  const double* avail;
  const int32_t* zone;
  const uint32_t* tb;
  const double* key;      // CA_FF: frozen per-group host key
  const double* dem;      // window tasks [nt][4]
  const int32_t* anc;     // window tasks [nt]
  const double* csum;
  const double* bsum;
  int H, Z, nt, S;        // S host segments: segment s = 64-host blocks s, s + S, ...
  int h_lo, h_hi;         // host range scored (a rank's shard; [0, H) unsharded)
  SegEntry* seg;          // [nt][S][KL]
  int32_t* seg_feas;      // [nt][S]
  int tw;                 // tasks per wave: 0 = the policy's default, else 2 or 4 (tuning/tests)
  const double* rtb;      // CA_BF realtime_bw: bandwidth per (group, host) [G][H], or NULL
  const int32_t* grp;     // window tasks' groups [nt] (rows of rtb)
};

// Merge of S sorted candidate lists per task into the task's exact top list. Two sources:
//   score segments   seg[(task*S + g)*KL + e], SL = KL, seg_feas[task*S + g] = feasible hosts
//                    of the segment (a list with more than KL of them is bounded by entry KL-1)
//   rank packages    (host-dimension sharding) seg[(g*nt + task)*(SL+1) + e]: SL entries then
//                    an explicit bound entry (id 0x7fffffff: the rank's list is complete);
//                    seg_feas = NULL
struct MergeArgs {
  const SegEntry* seg;
  const int32_t* seg_feas;
  const double* avail;
  const int32_t* zone;
  const double* dem;      // window tasks [nt][4]
  const int32_t* anc;     // window tasks [nt]
  const int32_t* ord;     // window tasks' caller indices
  int H, nt, S;
  int SL;                 // entries per source list (KL, or the package depth)
  Lists L;
  const int32_t* nt_dev;  // or NULL: only tasks [0, *nt_dev) (vbp best-fit representative lists)
  int bitonic;            // 1: the bitonic merge_kernel always (A/B; PVT_MERGE_SMALL=0 at ctx create)
  const int32_t* gate;    // or NULL: enqueued-ahead window (gate_closed below)
};

// Host-dimension sharding: a rank's exact local lists -> its exchange package (see MergeArgs).
struct PackArgs {
  Lists L;                // local merged lists of the window
  int nt, PK;
  int ordered;            // index-order first-fit lists (score 0, bound = last id + 1)
  SegEntry* out;          // [nt][PK + 1]
};

struct OrderedArgs {      // first-fit by host index: first KL snapshot-feasible hosts
  const double* avail;
  const int32_t* zone;
  const double* dem;
  const int32_t* anc;
  const int32_t* ord;
  int H, nt, strict;
  int h_lo, h_hi;         // host range scanned
  Lists L;
};

// One walked task of an epoch walk (chain mode): its winner's key (score, host; id -1 = no
// host) and the host's capacities after the commit; sup = 1 once a later task of the same
// group segment committed to the same host (the entry is then not the segment's final state).
struct WinRec {
  double s;
  int32_t id;
  int32_t sup;
  double a[4];
};

struct CommitArgs {
  double* avail;          // global state, updated in place
  const double* dem;      // window tasks [nt][4] (for the window's minimum demand)
  const double* csum;
  const double* bsum;
  const int32_t* zone;    // host zones / tiebreak ranks (for inherited touched hosts)
  const uint32_t* tb;     //   tb may be NULL (rank 0 for every host)
  Lists L;
  int H, Z, nt, mode;
  int32_t* placement;     // [T] in caller order
  // Hosts committed to by the previous window whose list entries in THIS window are stale
  // (the lists were scored before that window's commits landed): treated as touched.
  const int32_t* prev_ids;
  int n_prev;
  int32_t* own_ids;       // out: hosts this walk committed to (distinct), for the next window
  int32_t* status;        // out: [0] window-local index where the walk stopped (nt = done,
                          //      -1 = spin timeout), [1] number of own_ids
  const double* rtb;      // CA_BF realtime_bw: bandwidth per (group, host) [G][H], or NULL
  const int32_t* grp;     // window tasks' groups [nt] (rows of rtb)
  uint64_t* stamps;       // diagnostic builds only (PVT_STAMPS): per-phase cycle sums
  // Speculative epochs (pvt_capi.hip place_epochs), chain mode when cmap is set: workgroup b
  // walks the window tasks cmap[coff[b] .. coff[b+1]) (processing order), a chain of group
  // segments whose chain-local starts are cseg[csoff[b] .. csoff[b+1]); it writes wlog[w] for
  // every walked window task w instead of avail, and status[2b] = tasks walked.
  const int32_t* coff;
  const int32_t* cmap;
  const int32_t* csoff;
  const int32_t* cseg;
  WinRec* wlog;
  int skip_done;          // chain mode: a chain whose status already says "all walked" is skipped
  // vbp best-fit representative lists (pvt_band.hip band_runs_kernel): window task w's list is row
  // rowmap[w], its caller index ordw[w] (the list rows' TaskRec.ord belong to other tasks);
  // NULL: row w, TaskRec.ord
  const int32_t* rowmap;  //   (row = rowmap[w] - rowbase: the round's run ids, band_runs_kernel)
  const int32_t* ordw;
  // Windows enqueued ahead (pvt_capi.hip place_ahead; one-wave list walk only): gate = the walk
  // before's status slot {stopped at, owned hosts, nt, skipped} -- closed (gate_closed) when that
  // walk was skipped or stopped early: this walk is skipped (status {0, 0, nt, 1}); open: its
  // owned hosts are this walk's inherited ones (n_prev). ahead: status is such a 4-word slot.
  const int32_t* gate;
  int ahead;
  int rowbase;
  // or NULL: mapped pinned words the walk also reports to -- [1] = status[0], [2] = status[1],
  // then [0] = hseq (system-scope release): the host polls them instead of a copy + sync
  int32_t* hflag;
  int32_t hseq;
};

// Speculative epochs, cost_aware best-fit. The epoch's group segments (processing order,
// contiguous window ranges seg_off) are walked in chains -- the segments whose anchors share a
// zero-cost zone component, in order, by one workgroup -- all chains side by side on the epoch's
// start state. Segment j is exact iff every earlier segment is exact and complete, and for
// every task t it walked and every final log entry (host h, capacities after that segment) of
// an earlier segment of ANOTHER chain: h is not t's winner and h does not fit t with a key
// (score, index) below the winner's.
struct EpochArgs {
  const double* dem;      // window tasks [nt][4]
  const int32_t* anc;     // window tasks [nt]
  const double* csum;
  const double* bsum;
  const int32_t* zone;
  const int32_t* seg_off; // [nseg + 1] window offsets of the segments (processing order)
  const int32_t* seg_chain;   // [nseg] chain of each segment
  const int32_t* seg_cstart;  // [nseg] index of the segment's first task in its chain's walk
  const int32_t* status;  // [nchains][2]: tasks the chain's walk got through (-1: timeout)
  WinRec* wlog;           // [nt] (sup set by the finality pass)
  double* avail;          // apply: accepted segments' final entries written here
  int H, Z, nt, nseg;
  int32_t* bad;           // [nseg] out: 1 = segment j is not exact (zeroed by the caller)
  const double* rtb;      // realtime_bw: bandwidth per (group, host) [G][H], or NULL
  const int32_t* grp;     // window tasks' groups [nt]
  int whole;              // accept: whole segments only (first-fit zero-key epochs)
  // frontier-walked epochs (cost_aware best-fit): when every chain was walked to its end by the
  // zero-cost frontier walk and every final log entry exceeds the epoch's largest demand by
  // 2^-287 in some dimension (safe[j], set by the finality pass from the chains' cmax), no pair
  // can beat a winner (hosts of different components, scores > 0) and validation is skipped
  const double* cmax;     // [nch][4] or NULL
  const int32_t* coff;    // [nch + 1] chains' task ranges (their lengths)
  int nch;
  int32_t* safe;          // [nseg]
};
void launch_epoch_validate(const EpochArgs& a, hipStream_t st);
// finality only (no pair validation: first-fit zero-key epochs)
void launch_epoch_final(const EpochArgs& a, hipStream_t st);
// apply: the accepted segments [0, n_accept) of each chain, chain by chain in segment order
void launch_epoch_apply(const EpochArgs& a, int n_accept, int nchains, hipStream_t st);
// validate's verdict to the accepted prefix and its apply, on the device; res[5] reported, and
// (hout: mapped pinned memory) the nwords readback words from a.status copied there
void launch_epoch_accept_apply(const EpochArgs& a, int32_t* res, int nchains, hipStream_t st,
                               int32_t* hout = nullptr, int nwords = 0);
void launch_commit_chains(const CommitArgs& a, int nchains, hipStream_t st);
// vbp best-fit windows: the one-wave list walk with list cursors (pvt_lwalk.hip); CommitArgs as
// for launch_commit (no epochs, no stamps). status[0] < nt: refill there (0: the list walk decides)
void launch_lwalk(const CommitArgs& a, hipStream_t st);
hipError_t lwalk_init_attrs();

// Zero-cost frontier walk of epoch chains (pvt_zwalk.hip): workgroup b walks chain b like the
// list walk's chain mode (same tables, WinRec log, status[2b] = tasks walked) while it can prove
// every winner is the lowest-index fitting zero-cost host of its window; otherwise it writes
// status[2b] = -2 and leaves the chain to the list walk (CommitArgs.skip_done).
// An epoch's chain tables passed BY VALUE in the frontier walk's kernel arguments (instead of an
// upload launch before the walk: ~4 us of kernel plus its dispatch gap on the default line).
// Segment k (one group's tasks in the epoch, processing order): epoch tasks [seg_off[k],
// seg_off[k + 1]), walked by chain seg_chain[k] from chain-local position seg_cstart[k]. Chain c:
// chain-local positions [0, coff[c + 1] - coff[c]), its segments csegid[csoff[c] .. csoff[c+1]) in
// order. The walk's block 0 writes seg_off / seg_chain / seg_cstart / coff to the out pointers for
// the epoch kernels after it. nch = 0: the tables come from the device arrays (ZwalkArgs.coff ...).
constexpr int CT_SEGS = 64;
struct ChainTab {
  int32_t nseg, nch;
  int32_t seg_off[CT_SEGS + 1];
  int32_t seg_chain[CT_SEGS];
  int32_t seg_cstart[CT_SEGS];
  int32_t coff[CT_SEGS + 1];
  int32_t csoff[CT_SEGS + 1];
  int32_t csegid[CT_SEGS];
  int32_t* o_seg_off;
  int32_t* o_seg_chain;
  int32_t* o_seg_cstart;
  int32_t* o_coff;
};
struct ZwalkArgs {
  const double* avail;    // epoch-start capacities [4][H]
  const int32_t* zone;
  int H, Z;
  const double* dem;      // window tasks [nt][4]
  const int32_t* anc;     // window tasks' anchors
  const int32_t* ord;     // window task -> caller index (placement)
  const double* csum;
  const double* bsum;
  const int32_t* coff;
  const int32_t* cmap;
  int32_t* status;
  WinRec* wlog;
  int32_t* placement;
  const double* hmin;     // per-dimension host minima, launch_host_min partials
  uint64_t* stamps;       // diagnostic builds only (PVT_STAMPS)
  // keyed first-fit mode (launch_zwalk_keyed): one group of knt tasks, window = the first hosts
  // of the zero-key prefix kperm[0, kn) (+ lo), capacities written back to wb at the end
  const int32_t* kperm;
  int kn, lo, knt;
  double* wb;
  const int32_t* kn_dev;  // keyed: prefix length read on the device (NULL: kn)
  // host-sharded rounds: the merged window of chain b (keyed / ordered: of the walk) -- hosts
  // in index order with their capacities, as the unsharded walk builds it -- or NULL (build it)
  const struct FrontierSlot* pwin;
  // chain mode: chain b's group segments start at chain-local positions cseg[csoff[b] ..
  // csoff[b+1]) (a run of equal demands never crosses one: finality and apply work per
  // segment, so every segment's last copy on a host must be logged); NULL in keyed mode
  const int32_t* csoff;
  const int32_t* cseg;
  double* cmax;           // chain mode: [chains][4] out, each chain's largest demand per dimension
  // chain mode, the round's first epoch: windows the grouped order's launch built from the
  // snapshot (a chain uses the one whose zone set covers its anchors' zero-cost zones), or NULL
  const struct ZoneWindows* zpre;
  ChainTab tab;           // chain mode: the epoch's chain tables by value (tab.nch > 0), or none
};
constexpr int ZW_MIN_PARTS = 256;
// per-dimension minima of avail over hosts [lo, hi) into part[ZW_MIN_PARTS][4]
void launch_host_min(const double* avail, int H, int lo, int hi, double* part, hipStream_t st);
void launch_zwalk(const ZwalkArgs& a, int nchains, hipStream_t st);
// the same walk over a window of ZW_MBIG hosts (status[1] == 2: a chain's window of ZW_M was
// exhausted while more of its zones' hosts exist -- config 5 with loaded hosts)
void launch_zwalk_big(const ZwalkArgs& a, int nchains, hipStream_t st);
// cost_aware first-fit with sort_hosts: the zero-key chain walk (FF mode; hmin = the
// launch_host_absmax partials)
void launch_zwalk_ff(const ZwalkArgs& a, int nchains, hipStream_t st);
void launch_host_absmax(const double* avail, int H, int lo, int hi, double* part, hipStream_t st);
constexpr int ZW_M = 1024;                 // frontier-walk window hosts
void launch_zwalk_keyed(const ZwalkArgs& a, bool strict, hipStream_t st);
// ordered first-fit frontier: flags[h - lo] = host h in [lo, hs) fits the smallest demand of
// tasks dem[0, n)
void launch_alive_flags(const double* avail, int H, int lo, int hs, const double* dem, int n,
                        int strict, double* dmin, uint8_t* flags, hipStream_t st);

// Host-sharded frontier walks (pvt_capi.hip pvt_shard_*). A rank's package carries, per chain
// (cost_aware best-fit epochs) or for the one keyed / ordered walk, the first ZW_M window hosts
// of ITS host range in index order with their capacities, plus its host minima (certificate 2).
// After the all-gather every rank merges the packages -- ranks own ascending contiguous ranges,
// so the concatenation in rank order truncated to ZW_M is the window the unsharded walk builds
// -- and runs the same walk on identical inputs.
struct FrontierSlot {
  int32_t n;              // window hosts listed (<= ZW_M)
  int32_t total;          // candidates counted in the range (ordered walk: alive hosts)
  int32_t pad[2];
  int32_t id[ZW_M];       // global host index, ascending
  double a[4][ZW_M];      // capacities
};
// Zero-cost windows prebuilt by the grouped order's launch (group_sort_gather_kernel) for the
// round's first epoch of cost_aware best-fit: for each zone j that is the lowest zone of its
// zero-cost component (zones joined by csum = 0), U[j] = the union of the zero-cost zones of the
// round's group anchors in that component, and w[j] the first ZW_M hosts of U[j] in index order
// with their zones and snapshot capacities (bad: some capacity is not finite with |x| <= 2^500,
// certificate 3). U[j] = 0: no window for j. A chain's U (its anchors' zero-cost zones) lies in
// one component, so it is covered by that component's U[j]; a window over a superset of the
// zones is exact for the walk (pvt_zwalk.hip certificates).
struct ZoneWindow {
  int32_t n, bad, pad[2];
  int32_t id[ZW_M];
  int32_t z[ZW_M];
  double a[4][ZW_M];
};
struct ZoneWindows {
  uint32_t U[ZMAX];
  ZoneWindow w[ZMAX];
};
struct FrontierHdr {
  int32_t kind, nslots, pad[14];
  double hmin[ZW_MIN_PARTS][4];   // host-minimum partials over the rank's range
};
struct ZwinArgs {         // window candidates of one rank, per epoch chain
  const double* avail;
  const int32_t* zone;
  int H, Z, lo, hi;
  const double* csum;
  const int32_t* anc;     // epoch tasks' anchors
  const int32_t* coff;    // chain c: epoch tasks cmap[coff[c] .. coff[c+1])
  const int32_t* cmap;
  FrontierSlot* out;      // [nchains]
};
void launch_zwin_build(const ZwinArgs& a, int nchains, hipStream_t st);
// keyed / ordered walks: slot from a compacted local host list (host lo + perm[p], p < *count)
void launch_zwin_gather(const double* avail, int H, int lo, const int32_t* perm,
                        const int32_t* count, FrontierSlot* out, hipStream_t st);
// after the all-gather: merged slots [nslots] and host-minimum partials (ZW_MIN_PARTS x 4)
void launch_zwin_merge(const uint8_t* pkgs, int64_t pkg_bytes, int world, int nslots,
                       FrontierSlot* out, double* hmin, hipStream_t st);

// cost_aware first-fit with sort_hosts, as the reference runs it (cost_aware.py:118-124): the
// hosts sorted once per group by the frozen key (perm, skey = sorted key bits; the radix sort
// is stable, so equal keys keep host order), then per task the first `depth` snapshot-feasible
// hosts in that order. Lists come out exactly as merge_kernel would build them: sorted by
// (key, 0, host), cnt, complete, and a bound every unlisted host ranks at or after.
struct PermArgs {
  const double* avail;
  const int32_t* zone;
  const uint64_t* skey;   // [n] sorted key bits
  const int32_t* perm;    // [n] host at each sorted position, minus h_lo
  const double* dem;      // window tasks [nt][4]
  const int32_t* anc;
  const int32_t* ord;
  int H, nt, n, depth;    // depth <= LMAX
  int h_lo;               // first host of the sorted range (a rank's shard; 0 unsharded)
  int partial;            // perm is a prefix of the order: every other host's key >= rest_s
  double rest_s;
  Lists L;
};

struct KeyArgs {          // CA_FF sort_hosts: key[h] = c*df / (||avail_h|| * bw)
  const double* avail;
  const int32_t* zone;
  const int32_t* decay;
  const double* csum;
  const double* bsum;
  int H, Z, anchor;
  int h_lo, h_hi;         // hosts whose key is computed
  double* key;
  const double* rtb;      // realtime_bw: the group's bandwidth row [H], or NULL
};

// vbp best-fit lists by a memory band (pvt_band.hip): hosts [lo, hi) sorted once per round by
// snapshot memory (sorted copy of their snapshot state), plus the hosts committed to since
// (touched: flags[H], list, count), scanned with their live state.
struct BandArgs {
  const uint64_t* key;    // [n] orderable bits of the snapshot avail[1], ascending
  const double* sa;       // [4][n] snapshot capacities in sorted order
  const uint32_t* stb;    // [n] host-id ranks in sorted order
  const int32_t* sid;     // [n] host index at each sorted position
  int n, lo, hi;          // sorted hosts = [lo, hi)
  const uint8_t* touched; // [H] 1: committed to since the snapshot
  const int32_t* tlist;   // touched hosts
  const int32_t* tcount;  // [1]
  const double* avail;    // live state [4][H]
  const uint32_t* tb;     // [H]
  int H;
  const double* dem;      // window tasks [nt][4]
  int nt, S;              // S list segments per task
  SegEntry* seg;          // [nt][S][KL]
  int32_t* seg_feas;      // [nt][S]
  const int32_t* nt_dev;  // or NULL: only tasks [0, *nt_dev) (representative lists)
  const uint8_t* ptouched;  // [n] touched by sorted position (= touched[sid[p]], read with the chunk)
  const int32_t* gate;    // or NULL: enqueued-ahead window (gate_closed)
};

// An enqueued-ahead window's gate: the status slot {stopped at, owned hosts, nt, skipped} of the
// walk two windows back for the lists (one back for a walk): closed when that walk was skipped
// or stopped early -- the window was speculated on a continuation that did not happen.
__device__ __forceinline__ bool gate_closed(const int32_t* g) {
  if (!g) return false;
  const int s = __builtin_amdgcn_readfirstlane(g[3]), a = __builtin_amdgcn_readfirstlane(g[0]);
  const int n = __builtin_amdgcn_readfirstlane(g[2]);
  return s != 0 || a != n;
}
// A host's snapshot row for the band sort's gather (one 64-byte line per host).
struct alignas(64) BandRec {
  double a[4];
  uint32_t tb;
  uint32_t pad[7];
};
// sort keys and host records (rec[p] for host lo + p)
void launch_band_keys(const double* avail, const uint32_t* tb, int H, int lo, int n, uint64_t* key,
                      int32_t* idx, BandRec* rec, hipStream_t st);
void launch_band_gather(const BandRec* rec, int lo, int n, const int32_t* sid, double* sa,
                        uint32_t* stb, int32_t* pos, hipStream_t st);
void launch_touch_update(const int32_t* own, const int32_t* status, uint8_t* flags, int32_t* tlist,
                         int32_t* tcount, const int32_t* pos, int lo, int hi, uint8_t* ptouch,
                         hipStream_t st);
void launch_band_score(const BandArgs& a, hipStream_t st);
// Window tasks -> list rows: each run of equal demand vectors (bit for bit) shares one list row;
// rdem = the rows' demands, *nrep = rows (nt <= MAX_WINDOW)
void launch_band_runs(const double* dem, int T, int32_t* run, double* rdem, hipStream_t st);

int score_tasks_per_wave(int mode, int hosts, int force = 0);
int score_diag(uint64_t* out, int n, int reset);   // PVT_DIAG builds; else PVT_EUNSUPPORTED
void launch_score(int mode, const ScoreArgs& a, hipStream_t st);
void launch_merge(const MergeArgs& a, hipStream_t st);
const char* merge_kernel_name(const MergeArgs& a);   // the kernel launch_merge picks
void launch_pack(const PackArgs& a, hipStream_t st);
void launch_ordered(const OrderedArgs& a, hipStream_t st);
void launch_perm_scan(const PermArgs& a, hipStream_t st);
void launch_zero_key_flags(const double* key, int n, uint8_t* flags, hipStream_t st);
void launch_commit(const CommitArgs& a, hipStream_t st);
void launch_key(const KeyArgs& a, hipStream_t st);
void launch_zone_tables(const double* cost, const double* bw, int Z, double* csum, double* bsum,
                        hipStream_t st);
// a2: u64 sort key ~bits(||d||2) per task (descending norm == ascending key)
void launch_norm_keys(const double* dem, int T, const int32_t* idx, uint64_t* keys,
                      hipStream_t st);
void launch_group_keys(const int32_t* task_group, const int32_t* idx, int T, uint32_t* keys,
                       hipStream_t st);
// Resident rounds (pvt_batch.hip): one block per round (1 wave up to 1024 hosts, else 4), hosts
// in registers (HPL hosts per lane, HPL in {1, 2, 4, 8, 16}).
constexpr int RES_THREADS = 256;
constexpr int RES_MAX_HPL = 16;
constexpr int RES_MAX_HOSTS = RES_THREADS * RES_MAX_HPL;   // 4096
constexpr int RES_MAX_TASKS = 4096;
constexpr int RES_MIXED = -1;   // launch_resident: rounds of different policies (4 waves)
struct ResidentArgs {
  const void* rounds;     // device copy of pvt_round[n] (device array pointers)
  uint32_t* mt;           // [n][625] MT19937 states (PVT_OPP; the kernel uses R.mt_state)
  int Zb;                 // zone-table stride in LDS: max n_zones of the batch
  int Tpad;               // power of two >= max n_tasks of the batch (sort network size)
  uint64_t* stamps;       // diagnostic builds only (PVT_STAMPS): block 0 wave 0 phase cycles
  int walk = 0;           // 1: rounds of <= RW_MAXH hosts start with the one-wave resident walk
};
constexpr int RW_MAXH = 1024;   // resident walk: hosts held in LDS
size_t resident_lds_bytes(int Zb, int Tpad, bool walk);
void resident_shape(int maxH, int* waves, int* hpl);
void launch_resident(int mode, int waves, int hpl, int n, const ResidentArgs& a, hipStream_t st);
hipError_t resident_init_attrs();

// The fused host batch (pvt_place_host_batch): per round (one workgroup of four waves), its byte
// ranges of the pinned stage -- the same offsets in the mapped host copy and the device copy --
// and its index in the stage's AnchorArgs / CaGroupArgs arrays (-1: no fused grouping).
struct FusedRound {
  int64_t out_lo, out_hi, in_lo, in_hi;
  int64_t desc;           // byte offset of its pvt_round (device array pointers)
  int32_t items, pad;
};
struct FusedArgs {
  const char* hmap;       // the mapped pinned stage (the device reads its inputs, writes results)
  char* dev;              // the device copy of the stage
  int64_t o_rounds;       // FusedRound[n] (read from hmap)
  int64_t o_ka, o_kg;     // AnchorArgs[ni], CaGroupArgs[ni] (read from hmap)
  ResidentArgs ra;        // Zb, Tpad, walk, stamps (rounds unused: each workgroup has its own)
};
size_t fused_pre_lds_bytes();   // LDS of the anchor and grouping phases
void launch_fused(int mode, int hpl, int n, size_t lds, const FusedArgs& F, hipStream_t st);
size_t commit_lds_bytes();
hipError_t init_kernel_attrs();
// grouped processing order: group counts (cnt[G] = out-of-range ids), scatter by group, one
// LDS bitonic sort of (key, task index) per group of at most GSORT_MAX tasks
constexpr int GSORT_MAX = 4096;
void launch_group_hist(const int32_t* tg, int T, int G, int32_t* cnt, hipStream_t st);
// the grouped order's preparation in one block (T <= PREP_T_MAX, G <= GAGG_MAX): placement fill,
// group counts, pinned staging, offsets, zone tables, sort keys and the (key, task) scatter
constexpr int PREP_T_MAX = 65536;
constexpr int GAGG_MAX = 4096;
struct PrepArgs {
  const int32_t* tg;
  int T, G;
  const int32_t* ganc;
  const double* cost;
  const double* bw;
  int Z, nz2;                 // nz2: entries of the cost table staged (0: none)
  const double* dem;
  int sort_tasks;
  int32_t* placement;         // filled with -1, or NULL
  int32_t* off;               // [G + 1] group offsets in processing order
  int32_t* hcnt;              // pinned (device-mapped): counts [G + 1], anchors [G], cost [nz2]
  int32_t* hgan;
  double* hcst;
  double* csum;               // zone tables [Z * Z], or NULL
  double* bsum;
  uint64_t* skey;
  int32_t* sidx;
  int32_t* hflag;             // mapped pinned word, or NULL: order_count_kernel stores seq there
  int32_t seq;                //   once the staged counts are visible to the host
};
// counted (optional): recorded once the counts are staged, before the scatter launch (scatter
// = false: counts only, for launch_group_sort_gather)
void launch_order_prep(const PrepArgs& a, hipStream_t st, hipEvent_t counted = nullptr,
                       bool scatter = true);
// Few groups (G <= GCOMPACT_MAX): after the counts, one launch collects, sorts and gathers every
// group (order, caller order, demand rows, anchors, groups), fills placement and zone tables.
constexpr int GCOMPACT_MAX = 64;
struct GatherOut {
  int32_t* ord;
  double* dem_ord;
  int32_t* anc_ord;
  int32_t* grp_ord;
  int32_t* order_out;         // the caller's order, or NULL
  const double* avail;        // hmin != NULL: the same launch also writes the host minima over
  int H;                      //   [0, H) (ZW_MIN_PARTS partials as host_min_kernel's, one per
  double* hmin;               //   extra block)
  uint64_t* stamps;           // diagnostic builds only (PVT_STAMPS): block 0's phases, [16, 20)
  const int32_t* zone;        // zwin != NULL: Z more blocks prebuild the first epoch's zero-cost
  struct ZoneWindows* zwin;   //   windows from the snapshot (ZoneWindows), or NULL
};
void launch_group_sort_gather(const PrepArgs& a, const GatherOut& o, hipStream_t st);
// bytes (rounded up to 16; both buffers 16-B aligned and that long) from mapped pinned memory
void launch_upload(const void* src_mapped, void* dst, size_t bytes, hipStream_t st);
void launch_restore_hosts(double* avail, const double* avail0, int H, const int32_t* hosts, int n,
                          hipStream_t st);
void launch_group_stage(const int32_t* cnt, int G, const int32_t* ganc, const double* cost, int nz2,
                        int32_t* off, int32_t* hcnt, int32_t* hgan, double* hcst, hipStream_t st);
void launch_group_scatter(const int32_t* tg, const uint64_t* keys, int T, int G, int32_t* cursor,
                          uint64_t* skey, int32_t* sidx, hipStream_t st);
void launch_group_sort(const int32_t* off, int G, const uint64_t* skey, const int32_t* sidx,
                       int32_t* ord, hipStream_t st);
void launch_iota(int32_t* out, int n, hipStream_t st);
// gather tasks into processing order: dem_ord[p][r] = dem[r*T + ord[p]], anc_ord[p]
void launch_gather_tasks(const double* dem, const int32_t* ord, const int32_t* task_group,
                         const int32_t* group_anchor, int T, double* dem_ord, int32_t* anc_ord,
                         int32_t* grp_ord, hipStream_t st, int G = 0x7fffffff,
                         int32_t* order_out = nullptr);

}  // namespace pvt
