// group.h -- cross-rank statistic reduction (group.hip) used by bbtrain.hip.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/posfeat_hip.h"

int pf_group_world(const posfeat_group* g);
// in-place sum over the group's ranks of n doubles on stream st (no-op for
// a null group or world 1)
int pf_group_allreduce(posfeat_group* g, double* buf, int n, hipStream_t st);
