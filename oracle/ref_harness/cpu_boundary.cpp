// cpu_boundary.cpp -- TEST INFRASTRUCTURE (oracle/_ref only; never shipped).
//
// A CPU backend for the seven GPU symbols the reference's vector BinFHE code calls
// (SURVEY.md 8(b)), built ONLY from the reference's own CPU functions, so that the
// reference's unchanged vector path (binfhe-base-scheme.cpp:598-1277) can run in this
// container and produce golden vectors.  This is the contract SURVEY.md Appendix B
// validated ("Contract-validation probe"):
//   EvalAcc_CUDA   = per ciphertext: SetFormat(EVALUATION),
//                    RingGSWAccumulatorCGGI::EvalAcc(..., "NTT") (rgsw-acc-cggi.cpp:143-155),
//                    Transpose() of acc0 (the reference GPU returns it transposed,
//                    bootstrapping.cu:675-686), both polynomials back to COEFFICIENT;
//   MKMSwitch_CUDA = ModSwitch(qKS) -> KeySwitch -> ModSwitch(fmod) (lwe-pke.cpp:204-215,299-321),
//                    output NativeVector(n, fmod) (bootstrapping.cu:1898,1926);
//   CiphertextMulMatrix_CUDA: exact sum mod `modulus` of the reference formula
//                    (lwe-operation.cu:50-137, FP64 there: equal while sums < 2^53).
#include "binfhecontext.h"
#include "bootstrapping.cuh"
#include "lwe-operation.cuh"
#include "rgsw-acc-cggi.h"
#include "lwe-pke.h"

namespace lbcrypto {
namespace {
RingGSWACCKey g_bsk;
LWESwitchingKey g_ksk;
bool g_setup = false;
}  // namespace

void GPUFFTBootstrap::GPUSetup(const std::shared_ptr<BinFHECryptoParams> params, RingGSWACCKey BSkey,
                               LWESwitchingKey KSkey, int numGPUs) {
    g_bsk = BSkey;
    g_ksk = KSkey;
    g_setup = true;
}

void GPUFFTBootstrap::GPUClean() {
    g_bsk.reset();
    g_ksk.reset();
    g_setup = false;
}

void GPUFFTBootstrap::EvalAcc_CUDA(const std::shared_ptr<RingGSWCryptoParams> params,
                                   const std::vector<NativeVector>& a,
                                   std::shared_ptr<std::vector<RLWECiphertext>> acc, uint64_t fmod) {
    if (!g_setup)
        OPENFHE_THROW(openfhe_error, "cpu boundary: GPUSetup not called");
    RingGSWAccumulatorCGGI accum;
#pragma omp parallel for schedule(dynamic, 1)
    for (size_t s = 0; s < acc->size(); ++s) {
        std::vector<NativePoly> e = (*acc)[s]->GetElements();
        e[0].SetFormat(Format::EVALUATION);
        e[1].SetFormat(Format::EVALUATION);
        RLWECiphertext c = std::make_shared<RLWECiphertextImpl>(std::move(e));
        accum.EvalAcc(params, g_bsk, c, a[s], "NTT", 0);
        std::vector<NativePoly> r = c->GetElements();
        r[0] = r[0].Transpose();
        r[0].SetFormat(Format::COEFFICIENT);
        r[1].SetFormat(Format::COEFFICIENT);
        (*acc)[s] = std::make_shared<RLWECiphertextImpl>(std::move(r));
    }
}

void GPUFFTBootstrap::MKMSwitch_CUDA(const std::shared_ptr<LWECryptoParams> params,
                                     std::shared_ptr<std::vector<LWECiphertext>> ctExt, NativeInteger fmod) {
    if (!g_setup)
        OPENFHE_THROW(openfhe_error, "cpu boundary: GPUSetup not called");
    LWEEncryptionScheme lwe;
#pragma omp parallel for schedule(dynamic, 1)
    for (size_t s = 0; s < ctExt->size(); ++s) {
        auto c = lwe.ModSwitch(params->GetqKS(), (*ctExt)[s]);
        c = lwe.KeySwitch(params, g_ksk, c);
        (*ctExt)[s] = lwe.ModSwitch(fmod, c);
    }
}

std::shared_ptr<std::vector<LWECiphertext>> GPULWEOperation::CiphertextMulMatrix_CUDA(
    const std::shared_ptr<BinFHECryptoParams> params, const std::vector<LWECiphertext>& ct,
    const std::vector<std::vector<int64_t>>& matrix, uint64_t modulus) {
    const uint32_t n = params->GetLWEParams()->Getn();
    const size_t K = ct.size(), cols = matrix.empty() ? 0 : matrix[0].size();
    auto res = std::make_shared<std::vector<LWECiphertext>>(cols);
    const unsigned __int128 m = modulus;
    for (size_t c = 0; c < cols; ++c) {
        NativeVector av(n, modulus);
        __int128 b = 0;
        std::vector<__int128> acc(n, 0);
        for (size_t k = 0; k < K; ++k) {
            const __int128 w = matrix[k][c];
            for (uint32_t l = 0; l < n; ++l) acc[l] += w * (__int128)ct[k]->GetA()[l].ConvertToInt();
            b += w * (__int128)ct[k]->GetB().ConvertToInt();
        }
        for (uint32_t l = 0; l < n; ++l) {
            __int128 r = acc[l] % (__int128)m;
            av[l] = (uint64_t)(r < 0 ? r + (__int128)m : r);
        }
        __int128 rb = b % (__int128)m;
        (*res)[c] = std::make_shared<LWECiphertextImpl>(std::move(av), NativeInteger((uint64_t)(rb < 0 ? rb + (__int128)m : rb)));
    }
    return res;
}

void GPULWEOperation::GPUSetup(int) {}
void GPULWEOperation::GPUClean() {}

}  // namespace lbcrypto
