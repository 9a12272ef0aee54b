// sort_u64.hip -- local_sort<uint64_t> (the gfx950 bitonic tile engine of
// bitonic.h), in its own translation unit so the key types compile in parallel.
#include "bitonic.h"

namespace misort {
template hipError_t local_sort<uint64_t>(const uint64_t*, uint64_t*, int64_t, bool, uint64_t*, hipStream_t,
                                        LaunchHook*, const StageIO*, bool);
template hipError_t run_pass<uint64_t>(const uint64_t*, uint64_t*, int64_t, int, int, int, int, hipStream_t);
}  // namespace misort
