// runsk_fg6.hip -- the multi-way merge passes (runsk.hip) built a second time
// with 64-key fences: fuller chunks (a chunk holds at most (FM + K) * FG keys,
// so the fence slack K * FG halves) for twice the fences to plan with.  The
// planner picks this build for large sorts (mergek_fence_log2, kernels.hip).
#define MISORT_RUNSK_FGL 6
#define MISORT_RUNSK_FN(x) x##_fg6
#define MISORT_RUNSK_SECOND 1
// u64 chunks: 8896 keys (139 fences of 64; the 128-key build's 8832 is 69 of
// 128): k_mergek -5 us per 2^29 pass (profiles/r05/mergek/cap_ab.txt)
#ifndef MISORT_MK_CAP64
#define MISORT_MK_CAP64 8896
#endif
#include "runsk.hip"
