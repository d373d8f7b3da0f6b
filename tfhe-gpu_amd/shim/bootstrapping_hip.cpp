// bootstrapping_hip.cpp -- the OpenFHE side of the drop-in: GPUFFTBootstrap / GPULWEOperation
// (the reference's seven GPU symbols, bootstrapping.cuh:111-136, lwe-operation.cuh:49-62)
// implemented over the tfhe_hip C-ABI (include/tfhe_hip.h).
//
// A maintainer builds this file in place of src/binfhe/lib/bootstrapping.cu and
// src/binfhe/lib/lwe-operation.cu and links tfhe-gpu_amd/lib/libtfhe_hip.so; nothing else in
// src/binfhe changes -- the vector BinFHEScheme code (binfhe-base-scheme.cpp:598-1277) keeps
// building test vectors, extracting and chaining exactly as before.  oracle/Makefile.ref compiles
// it against the reference's own headers and links it with the reference's CPU objects
// (oracle/_ref/ref_dropin), which is how tests/test_gpu_dropin.py runs the unchanged reference
// vector API on the MI355X engine.
//
// Marshalling (the reference converts one ciphertext at a time on one host thread,
// bootstrapping.cu:1616-1667, 1875-1933): every conversion loop here is an OpenMP loop over
// ciphertexts, the flat staging arrays persist between calls (no 100 MB first-touch per call), and
// the engine stages them through pinned blocks.  EvalAcc recognises the accumulators that
// BootstrapGateCore / BootstrapFuncCore build (acc0 = 0, acc1 non-zero only at multiples of
// 2N/q, binfhe-base-scheme.cpp:1110-1138, 1163-1185) and sends only their q/2 test-vector
// words (tfhe_eval_acc_tv), which the device expands.  TFHE_SHIM_TIMING=1 prints the time of
// each phase to stderr.
#include "bootstrapping.cuh"
#include "lwe-operation.cuh"
#include "lwe-keyswitchkey.h"
#include "lwe-ciphertext.h"
#include "utils/exception.h"
#include "tfhe_hip.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace lbcrypto {
namespace {
tfhe_ctx* g_ctx = nullptr;  // process-global, like the reference's static device state (bootstrapping.cuh:142-159)

void check(tfhe_status s, const char* where) {
    if (s != TFHE_OK)
        OPENFHE_THROW(openfhe_error, std::string(where) + ": " + tfhe_status_string(s) + ": " + tfhe_last_error());
}

void need_setup(const char* where) {
    if (!g_ctx) OPENFHE_THROW(openfhe_error, std::string(where) + ": GPUSetup has not been called");
}

// grow-only flat staging (pages stay mapped between calls)
template <typename T>
T* stage(std::vector<T>& v, size_t words) {
    if (v.size() < words) v.resize(words);
    return v.data();
}
std::vector<uint64_t> g_a, g_acc, g_tv, g_ext, g_out;

struct Timer {
    const bool on;
    double t0;
    const char* what;
    static double now() {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
    }
    explicit Timer(const char* w) : on(std::getenv("TFHE_SHIM_TIMING") != nullptr), t0(now()), what(w) {}
    void lap(const char* phase, size_t B) {
        if (!on) return;
        const double t = now();
        std::fprintf(stderr, "[shim] %s %s B=%zu %.3f ms\n", what, phase, B, t - t0);
        t0 = t;
    }
};
}  // namespace

void GPUFFTBootstrap::GPUSetup(const std::shared_ptr<BinFHECryptoParams> params, RingGSWACCKey BSkey,
                               LWESwitchingKey KSkey, int numGPUs) {
    Timer tm("GPUSetup");
    const auto& L = params->GetLWEParams();
    const auto& R = params->GetRingGSWParams();
    tfhe_params p{};
    p.n = L->Getn();
    p.N = L->GetN();
    p.q = L->Getq().ConvertToInt();
    p.Q = L->GetQ().ConvertToInt();
    p.qKS = L->GetqKS().ConvertToInt();
    p.baseKS = L->GetBaseKS();
    p.baseG = R->GetBaseG();
    p.numDigitsToThrow = R->GetNumDigitsToThrow();
    check(tfhe_params_finish(&p), "tfhe_params_finish");
    // BSK -> [n][2][dG2][2][N] exactly as OpenFHE holds it (EVALUATION format): no INTT here (the
    // reference runs one per polynomial in KeyCopy_FFT, bootstrapping.cu:1112-1137); tfhe_setup_eval
    // uses OpenFHE's own root and bit-reversed order.
    std::vector<uint64_t> bsk((size_t)p.n * 2 * p.dG2 * 2 * p.N);
    bool eval_ok = true;
#pragma omp parallel for collapse(2) reduction(&& : eval_ok)
    for (uint32_t i = 0; i < p.n; ++i)
        for (uint32_t key = 0; key < 2; ++key)
            for (uint32_t row = 0; row < p.dG2; ++row)
                for (uint32_t poly = 0; poly < 2; ++poly) {
                    const NativePoly& c = (*(*BSkey)[0][key][i])[row][poly];
                    eval_ok = eval_ok && c.GetFormat() == Format::EVALUATION;
                    uint64_t* dst = bsk.data() + ((((size_t)i * 2 + key) * p.dG2 + row) * 2 + poly) * p.N;
                    for (uint32_t x = 0; x < p.N; ++x) dst[x] = c[x].ConvertToInt();
                }
    if (!eval_ok) OPENFHE_THROW(openfhe_error, "GPUSetup: BSK polynomial not in EVALUATION format");
    // KSK -> [N][baseKS][dKS][n+1], B at index n (the reference's device layout, bootstrapping.cu:961-975)
    const auto& A = KSkey->GetElementsA();
    const auto& B = KSkey->GetElementsB();
    std::vector<uint64_t> ksk((size_t)p.N * p.baseKS * p.dKS * (p.n + 1));
#pragma omp parallel for
    for (uint32_t i = 0; i < p.N; ++i)
        for (uint32_t j = 0; j < p.baseKS; ++j)
            for (uint32_t k = 0; k < p.dKS; ++k) {
                uint64_t* row = ksk.data() + (((size_t)i * p.baseKS + j) * p.dKS + k) * (p.n + 1);
                for (uint32_t l = 0; l < p.n; ++l) row[l] = A[i][j][k][l].ConvertToInt();
                row[p.n] = B[i][j][k].ConvertToInt();
            }
    tm.lap("flatten keys", 0);
    GPUClean();  // the reference grows its device list on a second GPUSetup (bootstrapping.cu:762); here it re-creates
    // numGPUs <= 0 or more than visible: every visible device, as the reference (bootstrapping.cu:736-739)
    check(tfhe_setup_eval(&g_ctx, &p, bsk.data(), ksk.data(), numGPUs), "tfhe_setup_eval");
    tm.lap("tfhe_setup_eval", 0);
}

void GPUFFTBootstrap::GPUClean() {
    if (g_ctx) tfhe_clean(g_ctx);
    g_ctx = nullptr;
}

void GPUFFTBootstrap::EvalAcc_CUDA(const std::shared_ptr<RingGSWCryptoParams> params,
                                   const std::vector<NativeVector>& a,
                                   std::shared_ptr<std::vector<RLWECiphertext>> acc, uint64_t /*fmod*/) {
    need_setup("EvalAcc_CUDA");
    Timer tm("EvalAcc");
    const size_t Bn = acc->size();
    if (Bn == 0) return;
    if (a.size() != Bn) OPENFHE_THROW(openfhe_error, "EvalAcc_CUDA: a and acc sizes differ");
    const uint32_t N = params->GetN(), n = a[0].GetLength();
    const uint64_t amod = a[0].GetModulus().ConvertToInt();
    const uint64_t factor = amod ? (2ull * N) / amod : 0;  // test-vector stride (binfhe-base-scheme.cpp:1120)
    const uint32_t tvlen = factor ? (uint32_t)(N / factor) : 0;
    uint64_t* fa = stage(g_a, Bn * n);
    uint64_t* ftv = stage(g_tv, Bn * (size_t)tvlen);
    // pass 1: a, and whether every accumulator is a COEFFICIENT test vector (acc0 = 0, acc1 zero off
    // the stride); the "GPU" mode of RingGSWAccumulatorCGGI::EvalAcc passes EVALUATION-format
    // accumulators (rgsw-acc-cggi.cpp:196-205), which take the general path below
    int sparse = factor >= 1 && (2ull * N) % amod == 0;
#pragma omp parallel for reduction(&& : sparse)
    for (size_t s = 0; s < Bn; ++s) {
        const NativeVector& as = a[s];
        for (uint32_t l = 0; l < n; ++l) fa[s * n + l] = as[l].ConvertToInt();
        if (!sparse) continue;
        const auto& e = (*acc)[s]->GetElements();
        if (e[0].GetFormat() != Format::COEFFICIENT || e[1].GetFormat() != Format::COEFFICIENT) {
            sparse = 0;
            continue;
        }
        const NativeVector& v0 = e[0].GetValues();
        const NativeVector& v1 = e[1].GetValues();
        bool ok = true;
        for (uint32_t x = 0; x < N && ok; ++x) {
            ok = v0[x].ConvertToInt() == 0 && (x % factor == 0 || v1[x].ConvertToInt() == 0);
            if (x % factor == 0) ftv[s * tvlen + x / factor] = v1[x].ConvertToInt();
        }
        sparse = sparse && ok;
    }
    tm.lap(sparse ? "marshal in (test vectors)" : "marshal in", Bn);
    uint64_t* fac = stage(g_acc, Bn * 2 * N);
    if (sparse) {
        check(tfhe_eval_acc_tv(g_ctx, Bn, fa, amod, ftv, tvlen, fac), "tfhe_eval_acc_tv");
    } else {
#pragma omp parallel for
        for (size_t s = 0; s < Bn; ++s)
            for (uint32_t j = 0; j < 2; ++j) {
                NativePoly c = (*acc)[s]->GetElements()[j];
                c.SetFormat(Format::COEFFICIENT);
                const NativeVector& v = c.GetValues();
                for (uint32_t x = 0; x < N; ++x) fac[(s * 2 + j) * N + x] = v[x].ConvertToInt();
            }
        check(tfhe_eval_acc(g_ctx, Bn, fa, amod, fac), "tfhe_eval_acc");
    }
    tm.lap("device", Bn);
    const auto polyParams = params->GetPolyParams();
    const NativeInteger Q = params->GetQ();
    // Results go into the accumulators' own coefficient vectors when this vector holds the only
    // reference and they have the shape of the result (the callers' fresh test vectors): no
    // allocation.  Otherwise new objects, as the reference does (bootstrapping.cu:1655-1664); the
    // replaced ones are released on this thread afterwards (freeing another thread's blocks from
    // the OpenMP workers serialises on the allocator).
    std::vector<RLWECiphertext> old(Bn);
#pragma omp parallel for
    for (size_t s = 0; s < Bn; ++s) {  // acc0 already transposed (bootstrapping.cu:675-686)
        RLWECiphertext& ct = (*acc)[s];
        bool reuse = ct.use_count() == 1;
        if (reuse) {
            const auto& e = ct->GetElements();
            for (uint32_t j = 0; j < 2 && reuse; ++j)
                reuse = e[j].GetFormat() == Format::COEFFICIENT && e[j].GetLength() == N && e[j].GetModulus() == Q;
        }
        if (reuse) {
            auto& e = ct->GetElements();
            for (uint32_t j = 0; j < 2; ++j) {
                NativeVector& v = const_cast<NativeVector&>(e[j].GetValues());
                const uint64_t* src = fac + (s * 2 + j) * N;
                for (uint32_t x = 0; x < N; ++x) v[x] = src[x];
            }
            continue;
        }
        std::vector<NativePoly> res(2);
        for (uint32_t j = 0; j < 2; ++j) {
            NativeVector v(N, Q);
            const uint64_t* src = fac + (s * 2 + j) * N;
            for (uint32_t x = 0; x < N; ++x) v[x] = src[x];
            res[j] = NativePoly(polyParams, Format::COEFFICIENT, false);
            res[j].SetValues(std::move(v), Format::COEFFICIENT);
        }
        old[s] = std::move(ct);
        ct = std::make_shared<RLWECiphertextImpl>(std::move(res));
    }
    old.clear();
    tm.lap("marshal out", Bn);
}

void GPUFFTBootstrap::MKMSwitch_CUDA(const std::shared_ptr<LWECryptoParams> params,
                                     std::shared_ptr<std::vector<LWECiphertext>> ctExt, NativeInteger fmod) {
    need_setup("MKMSwitch_CUDA");
    Timer tm("MKMSwitch");
    const size_t Bn = ctExt->size();
    if (Bn == 0) return;
    const uint32_t N = params->GetN(), n = params->Getn();
    uint64_t* in = stage(g_ext, Bn * (N + 1));
    uint64_t* out = stage(g_out, Bn * (n + 1));
#pragma omp parallel for
    for (size_t s = 0; s < Bn; ++s) {
        const NativeVector& av = (*ctExt)[s]->GetA();
        for (uint32_t k = 0; k < N; ++k) in[s * (N + 1) + k] = av[k].ConvertToInt();
        in[s * (N + 1) + N] = (*ctExt)[s]->GetB().ConvertToInt();
    }
    tm.lap("marshal in", Bn);
    check(tfhe_mkm_switch(g_ctx, Bn, in, fmod.ConvertToInt(), out), "tfhe_mkm_switch");
    tm.lap("device", Bn);
    std::vector<LWECiphertext> old(Bn);  // released on this thread (see EvalAcc_CUDA)
#pragma omp parallel for
    for (size_t s = 0; s < Bn; ++s) {
        NativeVector av(n, fmod);  // output modulus fmod (bootstrapping.cu:1898,1926)
        for (uint32_t k = 0; k < n; ++k) av[k] = out[s * (n + 1) + k];
        old[s] = std::move((*ctExt)[s]);
        (*ctExt)[s] = std::make_shared<LWECiphertextImpl>(std::move(av), NativeInteger(out[s * (n + 1) + n]));
    }
    old.clear();
    tm.lap("marshal out", Bn);
}

std::shared_ptr<std::vector<LWECiphertext>> GPULWEOperation::CiphertextMulMatrix_CUDA(
    const std::shared_ptr<BinFHECryptoParams> params, const std::vector<LWECiphertext>& ct,
    const std::vector<std::vector<int64_t>>& matrix, uint64_t modulus) {
    need_setup("CiphertextMulMatrix_CUDA");
    const uint32_t n = params->GetLWEParams()->Getn();
    const size_t K = ct.size(), cols = matrix.empty() ? 0 : matrix[0].size();
    if (matrix.size() != K)  // lwe-operation.cu:66-69
        OPENFHE_THROW(openfhe_error, "The number of rows of the matrix must be equal to the number of input ciphertexts.");
    std::vector<uint64_t> in(K * (n + 1)), out(cols * (n + 1));
    std::vector<int64_t> m(K * cols);
#pragma omp parallel for
    for (size_t k = 0; k < K; ++k) {
        for (uint32_t l = 0; l < n; ++l) in[k * (n + 1) + l] = ct[k]->GetA()[l].ConvertToInt();
        in[k * (n + 1) + n] = ct[k]->GetB().ConvertToInt();
        for (size_t c = 0; c < cols; ++c) m[k * cols + c] = matrix[k][c];
    }
    check(tfhe_ciphertext_mul_matrix(g_ctx, K, in.data(), cols, m.data(), modulus, out.data()),
          "tfhe_ciphertext_mul_matrix");
    auto res = std::make_shared<std::vector<LWECiphertext>>(cols);
#pragma omp parallel for
    for (size_t c = 0; c < cols; ++c) {
        NativeVector av(n, modulus);
        for (uint32_t l = 0; l < n; ++l) av[l] = out[c * (n + 1) + l];
        (*res)[c] = std::make_shared<LWECiphertextImpl>(std::move(av), NativeInteger(out[c * (n + 1) + n]));
    }
    return res;
}

void GPULWEOperation::GPUSetup(int numGPUs) { check(tfhe_lwe_gpu_setup(numGPUs), "tfhe_lwe_gpu_setup"); }
void GPULWEOperation::GPUClean() { check(tfhe_lwe_gpu_clean(), "tfhe_lwe_gpu_clean"); }

}  // namespace lbcrypto
