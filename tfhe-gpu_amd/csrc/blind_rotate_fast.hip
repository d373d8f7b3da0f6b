// blind_rotate_fast.hip -- specialised STD128-class blind rotation (placeholder:
// the generic LDS kernel serves every parameter set until this path lands).
#include "device_math.hpp"
#include "kernels.hpp"

namespace tfhe {

bool fast_path_supported(const BRParams&, int) { return false; }
size_t bsk_fast_bytes(const BRParams&) { return 0; }
hipError_t launch_pack_bsk_fast(const BRParams&, const void*, const void*, void*, hipStream_t) {
    return hipErrorNotSupported;
}
hipError_t launch_blind_rotate_fast(const BRParams&, const DevTables&, const void*, const uint64_t*, uint64_t,
                                    uint64_t*, size_t, hipStream_t) {
    return hipErrorNotSupported;
}

}  // namespace tfhe
