// blind_rotate_fast4_d6.hip -- the four-wavefront kernel at the logQ = 11 folded digit shape
// (6 digits of 5 bits, top digit eliminated) in a translation unit of its own, so that it is built
// with the default LLVM scheduler while blind_rotate_fast4.hip uses iterative-ilp (Makefile):
// this shape ran 29 % slower under iterative-ilp, the others 2-3 % faster (profiles/r02bh).
#define TFHE_FAST4_KERNEL_ONLY
#include "blind_rotate_fast4.hip"

namespace tfhe {

hipError_t launch_blind_rotate_fast4_d6(const f4::FastConst& K, uint32_t n, uint32_t loga, const int32_t* tabs4,
                                        const int32_t* bsk, const uint64_t* a, uint64_t* acc, size_t B, hipStream_t s) {
    auto kern = f4::k_blind_rotate_fast4<4, 1, 0, 7, 1, 1, 6, 5, 0, true>;
    const size_t lb = f4::lds_bytes(2, 1, 1);
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lb);
    hipLaunchKernelGGL(kern, dim3((unsigned)B), dim3(f4::TPC), lb, s, K, n, loga, tabs4, bsk, a, acc, (uint32_t)B,
                       nullptr);
    return hipGetLastError();
}

}  // namespace tfhe
