// pvt_opp.h — opportunistic policy kernels (reference scheduler/opportunistic.py:11-20).
//
// Per task the reference lists every host with np.all(r >= d) in cluster order, draws
// randomizer.choice(qualified) (= randint(0, n), no draw when n == 1) and commits. On the GPU:
//   count kernel   per window task, the snapshot feasibility bitmap of every chunk of OPP_CH
//                  hosts and the count of every super-chunk of OPP_SUP chunks (fit-mask pass)
//   commit walk    one workgroup: per range of OPP_R tasks, the draws (MT19937 randint(n) in
//                  LDS, n = snapshot count minus the touched hosts that stopped fitting) and
//                  the candidate hosts from the k-th feasible on are computed in parallel; one
//                  wave then verifies and commits them in task order (pvt_opp.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pvt {

constexpr int OPP_CH = 256;     // hosts per chunk
constexpr int OPP_SUP = 64;     // chunks per super-chunk (16384 hosts)
constexpr int OPP_TW = 8;       // tasks per wave in the count kernel
constexpr int OPP_MAXW = 256;   // tasks per window (commit-walk LDS holds 2 x OPP_MAXW touched hosts)
constexpr int OPP_WINDOW_DEFAULT = 256;   // sequential count / walk
constexpr int OPP_WINDOW_PIPE = 256;      // pipelined windows (round-4 sweep at config 5 with
                                          // the register-row walk: 96 11.3, 128 10.0, 192 9.7,
                                          // 256 9.6 ms; config 3: 128 1.22, 256 1.15 ms)

struct OppCountArgs {
  const double* avail;
  const double* dem;      // window tasks [nt][4]
  int H, nt, S, seg_q, nq, nsq, ldc;   // S, seg_q: set by launch_opp_count
  uint64_t* bm;           // [ldc][ldq][4] per-chunk feasibility bitmaps (bit = host), task-major
  int32_t* sc;            // [ldc][lds] super-chunk counts, task-major
  // super-chunks [sq_lo, sq_hi) are counted (a rank's share under host sharding; [0, nsq)
  // unsharded); chunk q lands at row position q - sq_lo * OPP_SUP of ldq, super-chunk Q at
  // Q - sq_lo of lds
  int sq_lo, sq_hi, ldq, lds;
};

// Host sharding: rank r's package (ldq = P_sq * OPP_SUP chunks and lds = P_sq super-chunks per
// task, super-chunks [r * P_sq, ...)) -> the full task-major tables of a window.
struct OppUnpackArgs {
  const uint8_t* recv;    // world packages, pkg_bytes each
  int64_t pkg_bytes;
  int world, nt, nq, nsq, P_sq, ldc;
  uint64_t* bm;           // [ldc][nq][4]
  int32_t* sc;            // [ldc][nsq]
};
void launch_opp_unpack(const OppUnpackArgs& a, hipStream_t st);

// A walk's touched hosts handed to the next window's walk (pipelined windows): the next
// window's count pass ran on the capacities the walk started from, so these hosts are touched
// relative to it. sb = capacity when this walk started (the next count's snapshot), ta = after.
struct OppTouched {
  int32_t n, pad[3];
  int32_t tid[OPP_MAXW];
  double sb[4][OPP_MAXW];
  double ta[4][OPP_MAXW];
};

struct OppCommitArgs {
  double* avail;
  const double* dem;      // window tasks [nt][4]
  const uint64_t* bm;
  const int32_t* sc;
  int H, nt, nq, nsq, ldc;
  int32_t* placement;     // window tasks' placements (caller order == processing order)
  uint32_t* mt;           // device MT19937 state: key[624], pos
  uint64_t* stamps;       // diagnostic builds only (PVT_STAMPS): per-phase cycle sums
  const OppTouched* in;   // previous walk's hosts (already applied to avail by
                          // launch_opp_apply): touched for this walk
  OppTouched* out;        // this walk's own hosts for the next walk (NULL: none)
  int writeback;          // write this walk's own hosts to avail at the end
  int32_t* fault;         // set to 1 + task (window-local) when a range's first task fails its
                          // verification: inconsistent counts / bitmaps (the host reports EHIP)
};

void launch_opp_count(const OppCountArgs& a, hipStream_t st);
void launch_opp_commit(const OppCommitArgs& a, hipStream_t st);
// Pipelined windows: the previous walk's commits (t->ta) written to global availability before
// the next walk starts; an event after it releases the count pass of the window after.
void launch_opp_apply(const OppTouched* t, double* avail, int H, hipStream_t st);
hipError_t opp_init_attrs();

}  // namespace pvt
