// runsk_fg6.hip -- the multi-way merge passes (runsk.hip) built a second time
// with 64-key fences: fuller chunks (a chunk holds at most (FM + K) * FG keys,
// so the fence slack K * FG halves) for twice the fences to plan with.  The
// planner picks this build for large sorts (mergek_fence_log2, kernels.hip).
#define MISORT_RUNSK_FGL 6
#define MISORT_RUNSK_FN(x) x##_fg6
#define MISORT_RUNSK_SECOND 1
#include "runsk.hip"
