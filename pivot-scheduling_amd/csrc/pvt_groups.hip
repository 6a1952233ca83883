// pvt_groups.hip — cost_aware grouping on the device (the drop-in round's single round trip,
// pvt_place_host with pvt_ca_items).
//
// Reference (scheduler/cost_aware.py:30-58): ready tasks are grouped in first-seen order by
//   ('storage', cluster.get_storage_by_locality(mode host's zone))  for tasks with predecessors,
//   ('app', task.application)                                       for source tasks,
// and the groups run in that order, an application group's anchor drawn as
// randomizer.choice(cluster.storage) when its turn comes (:37-39). The mode hosts come from the
// anchor kernels (pvt_anchor.hip) over the items' predecessor lists; this kernel turns them into
// task_group / group_anchor / n_groups for the placement that follows on the same stream:
//   key(t)     storage index s (< S) or S + application index (anchor_zone -1: no predecessors)
//   first[k]   the lowest task index with key k (LDS atomicMin)
//   group(k)   the number of keys whose first task comes before first[k]: a block scan of the
//              "first task of its key" flags in task order
//   draws      one MT19937 randint(0, S) per application group, in group order, by one wave
//              (numpy legacy RandomState.choice: masked rejection, no draw for S == 1)
// One workgroup: at most 16384 tasks, a few microseconds of work.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pivot_place.h"
#include "pvt_device.h"
#include "pvt_groups_dev.h"
#include "pvt_kernels.h"
#include "pvt_mt.h"

namespace pvt {

constexpr int GR_THREADS = 1024;

__global__ __launch_bounds__(GR_THREADS) void ca_groups_kernel(CaGroupArgs A) {
  __shared__ GroupLds L;
  ca_groups_round<GR_THREADS, GRP_MAX_TASKS>(A, L);
}

// Several rounds' groupings in one launch, one workgroup each (pvt_place_host_batch).
__global__ __launch_bounds__(GR_THREADS) void ca_groups_batch_kernel(const CaGroupArgs* A) {
  __shared__ GroupLds L;
  const CaGroupArgs a = A[blockIdx.x];
  ca_groups_round<GR_THREADS, GRP_MAX_TASKS>(a, L);
}

void launch_ca_groups(const CaGroupArgs& a, hipStream_t st) {
  PVT_LAUNCH(ca_groups_kernel, dim3(1), dim3(GR_THREADS), 0, st, a);
}
void launch_ca_groups_batch(const CaGroupArgs* args_dev, int n, hipStream_t st) {
  if (n > 0) PVT_LAUNCH(ca_groups_batch_kernel, dim3(n), dim3(GR_THREADS), 0, st, args_dev);
}

}  // namespace pvt
