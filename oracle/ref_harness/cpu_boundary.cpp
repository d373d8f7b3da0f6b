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
#include <cmath>
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

// CiphertextMulMatrix_CUDA with the reference's own semantics (lwe-operation.cu:50-137) on the CPU:
// A[K][n+1] and B[K][cols] converted to double (ConvertToDouble / static_cast<double>), C = A B^T as an
// FP64 product, fmod(C, modulus) (applyFmod, :42-48), each entry static_cast<uint64_t> into a
// NativeVector(n, modulus) and a NativeInteger without further reduction (:115-122).  The only freedom
// taken: cuBLAS's DGEMM summation order is unspecified, so the sum runs k = 0 .. K-1 in order (this
// file is compiled without FMA contraction); every sum below 2^53 is exact in any order.  Where the
// reference's outputs leave [0, modulus) (negative sums: fmod keeps the sign and the cast wraps) or
// round (|sums| >= 2^53), the HIP engine's exact integer product differs by design.
std::shared_ptr<std::vector<LWECiphertext>> GPULWEOperation::CiphertextMulMatrix_CUDA(
    const std::shared_ptr<BinFHECryptoParams> params, const std::vector<LWECiphertext>& ct,
    const std::vector<std::vector<int64_t>>& matrix, uint64_t modulus) {
    if (ct.empty()) OPENFHE_THROW(openfhe_error, "Input ciphertexts are empty.");
    if (matrix.empty()) OPENFHE_THROW(openfhe_error, "Input matrix is empty.");
    if (ct.size() != matrix.size())
        OPENFHE_THROW(openfhe_error, "The number of rows of the matrix must be equal to the number of input ciphertexts.");
    const uint32_t n = params->GetLWEParams()->Getn(), M = n + 1;
    const size_t K = ct.size(), cols = matrix[0].size();
    std::vector<double> hA(M * K), hB(K * cols);
    for (size_t i = 0; i < K; ++i) {
        const NativeVector& a = ct[i]->GetA();
        for (uint32_t j = 0; j < n; ++j) hA[M * i + j] = a[j].ConvertToDouble();
        hA[M * i + n] = ct[i]->GetB().ConvertToDouble();
    }
    for (size_t i = 0; i < K; ++i)
        for (size_t j = 0; j < cols; ++j) hB[cols * i + j] = static_cast<double>(matrix[i][j]);
    const double dm = static_cast<double>(modulus);
    auto res = std::make_shared<std::vector<LWECiphertext>>(cols);
#pragma omp parallel for schedule(static)
    for (size_t c = 0; c < cols; ++c) {
        std::vector<double> C(M, 0.0);
        for (size_t k = 0; k < K; ++k) {
            const double w = hB[cols * k + c];
            for (uint32_t j = 0; j < M; ++j) C[j] += hA[M * k + j] * w;
        }
        NativeVector av(n, modulus);
        for (uint32_t j = 0; j < n; ++j) av[j] = static_cast<uint64_t>(std::fmod(C[j], dm));
        NativeInteger b(static_cast<uint64_t>(std::fmod(C[n], dm)));
        (*res)[c] = std::make_shared<LWECiphertextImpl>(LWECiphertextImpl(std::move(av), b));
    }
    return res;
}

void GPULWEOperation::GPUSetup(int) {}
void GPULWEOperation::GPUClean() {}

}  // namespace lbcrypto
