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
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace lbcrypto {
namespace {
tfhe_ctx* g_ctx = nullptr;  // process-global, like the reference's static device state (bootstrapping.cuh:142-159)
uint32_t g_n = 0;           // LWE dimension n of the set-up context (EvalAcc_CUDA checks every a row against it)

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

// The u64 storage of a NativeVector: NativeIntegerT<uint64_t> is one uint64_t with no virtual
// members, and NativeVectorT keeps its elements in one std::vector (mubintvecnat.h:645-651), so
// the rows can be handed to the engine's staging as plain u64 arrays.
static_assert(sizeof(NativeInteger) == sizeof(uint64_t), "NativeInteger is not one 64-bit word");
const uint64_t* words(const NativeVector& v) { return reinterpret_cast<const uint64_t*>(&v[0]); }
uint64_t* words(NativeVector& v) { return reinterpret_cast<uint64_t*>(&v[0]); }
uint64_t* words(const NativeVector& v, int) { return const_cast<uint64_t*>(words(v)); }


// The ciphertext objects a call replaces (8192 RLWE / LWE objects and their coefficient vectors per
// batch) are released by one background thread, after the call has returned: freeing them on the
// caller's thread took 1.6-1.9 ms per 8192 (profiles/r03o), and from the OpenMP workers the frees
// of blocks another thread allocated serialise on the allocator.  One heap object, intentionally
// never destroyed (its thread is detached).  flush() waits until every queued batch is freed: GPUClean
// and an atexit handler call it, so no destructor of an OpenFHE object runs after exit() has begun
// tearing down OpenFHE's static parameter and allocator state.
class Reaper {
   public:
    static Reaper& get() {
        static Reaper* r = [] {
            auto* x = new Reaper();
            std::atexit([] { Reaper::get().flush(); });
            return x;
        }();
        return *r;
    }
    static void drop(std::vector<std::shared_ptr<void>>&& batch) {
        Reaper& r = get();
        {
            std::lock_guard<std::mutex> lk(r.m_);
            r.q_.push_back(std::move(batch));
            ++r.queued_;
        }
        r.cv_.notify_one();
    }
    void flush() {
        std::unique_lock<std::mutex> lk(m_);
        done_cv_.wait(lk, [&] { return freed_ == queued_; });
    }

   private:
    Reaper() { std::thread([this] { loop(); }).detach(); }
    void loop() {
        for (;;) {
            std::vector<std::shared_ptr<void>> b;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return !q_.empty(); });
                b = std::move(q_.front());
                q_.pop_front();
            }
            b.clear();
            {
                std::lock_guard<std::mutex> lk(m_);
                ++freed_;
            }
            done_cv_.notify_all();
        }
    }
    std::mutex m_;
    std::condition_variable cv_, done_cv_;
    std::deque<std::vector<std::shared_ptr<void>>> q_;
    uint64_t queued_ = 0, freed_ = 0;
};

template <typename T>
void release_later(std::vector<std::shared_ptr<T>>& objs) {
    std::vector<std::shared_ptr<void>> b;
    b.reserve(objs.size());
    for (auto& o : objs)
        if (o) b.emplace_back(std::move(o));
    objs.clear();
    if (!b.empty()) Reaper::drop(std::move(b));
}

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
    g_n = p.n;
    tm.lap("tfhe_setup_eval", 0);
    if (tm.on) {  // which devices and replication GPUSetup(numGPUs) ended with (tests/test_gpu_dropin.py)
        tfhe_info info{};
        if (tfhe_get_info(g_ctx, &info) == TFHE_OK)
            std::fprintf(stderr, "[shim] GPUSetup devices=%d replicate_method=%d\n", info.num_devices,
                         info.replicate_method);
    }
}

void GPUFFTBootstrap::GPUClean() {
    Reaper::get().flush();  // objects replaced by earlier calls are freed before the caller moves on
    if (g_ctx) tfhe_clean(g_ctx);
    g_ctx = nullptr;
    g_n = 0;
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
    const auto polyParams = params->GetPolyParams();
    const NativeInteger Q = params->GetQ();
    // pass 1: the rows of a (no copy: the staging narrows them from their own storage), and whether
    // every accumulator is a COEFFICIENT test vector (acc0 = 0, acc1 zero off the stride); the "GPU"
    // mode of RingGSWAccumulatorCGGI::EvalAcc passes EVALUATION-format accumulators
    // (rgsw-acc-cggi.cpp:196-205), which take the general path below
    std::vector<const uint64_t*> arows(Bn);
    uint64_t* ftv = stage(g_tv, Bn * (size_t)tvlen);
    int sparse = factor >= 1 && (2ull * N) % amod == 0, lens_ok = 1;
#pragma omp parallel for reduction(&& : sparse, lens_ok)
    for (size_t s = 0; s < Bn; ++s) {
        lens_ok = lens_ok && a[s].GetLength() == n;
        arows[s] = words(a[s]);
        if (!sparse) continue;
        const auto& e = (*acc)[s]->GetElements();
        if (e[0].GetFormat() != Format::COEFFICIENT || e[1].GetFormat() != Format::COEFFICIENT ||
            e[0].GetLength() != N || e[1].GetLength() != N) {
            sparse = 0;
            continue;
        }
        const uint64_t* v0 = words(e[0].GetValues());
        const uint64_t* v1 = words(e[1].GetValues());
        uint64_t nz = 0;
        for (uint32_t x = 0; x < N; ++x) nz |= v0[x];
        for (uint32_t x = 0; x < N; x += (uint32_t)factor) {
            ftv[s * tvlen + x / factor] = v1[x];
            for (uint32_t y = x + 1; y < x + factor; ++y) nz |= v1[y];
        }
        sparse = sparse && nz == 0;
    }
    // the engine reads n words per row (the n of GPUSetup): shorter rows would be read past their end
    if (!lens_ok || n != g_n)
        OPENFHE_THROW(openfhe_error, "EvalAcc_CUDA: every a vector must have the LWE dimension n of GPUSetup (" +
                                         std::to_string(g_n) + ")");
    tm.lap(sparse ? "marshal in (test vectors)" : "marshal in", Bn);
    if (sparse) {
        // Results go into the accumulators' own coefficient vectors when this vector holds the only
        // reference and they have the shape of the result (the callers' fresh test vectors): the
        // staging writes them in place.  Otherwise into new objects, as the reference does
        // (bootstrapping.cu:1655-1664); the replaced ones go to the Reaper.
        std::vector<uint64_t*> rows(2 * Bn);
        std::vector<RLWECiphertext> fresh(Bn);
#pragma omp parallel for
        for (size_t s = 0; s < Bn; ++s) {
            RLWECiphertext& ct = (*acc)[s];
            bool reuse = ct.use_count() == 1;
            if (reuse) {
                const auto& e = ct->GetElements();
                for (uint32_t j = 0; j < 2 && reuse; ++j)
                    reuse = e[j].GetFormat() == Format::COEFFICIENT && e[j].GetLength() == N && e[j].GetModulus() == Q;
            }
            RLWECiphertext& dst = reuse ? ct : fresh[s];
            if (!reuse) {
                std::vector<NativePoly> res(2);
                for (uint32_t j = 0; j < 2; ++j) {
                    res[j] = NativePoly(polyParams, Format::COEFFICIENT, false);
                    res[j].SetValues(NativeVector(N, Q), Format::COEFFICIENT);
                }
                dst = std::make_shared<RLWECiphertextImpl>(std::move(res));
            }
            for (uint32_t j = 0; j < 2; ++j) rows[2 * s + j] = words(dst->GetElements()[j].GetValues(), 0);
        }
        tm.lap("output rows", Bn);
        check(tfhe_eval_acc_tv_rows(g_ctx, Bn, arows.data(), amod, ftv, tvlen, rows.data()),
              "tfhe_eval_acc_tv_rows");  // acc0 already transposed (bootstrapping.cu:675-686)
        tm.lap("device", Bn);
        for (size_t s = 0; s < Bn; ++s)
            if (fresh[s]) std::swap((*acc)[s], fresh[s]);
        release_later(fresh);
        tm.lap("marshal out", Bn);
        return;
    }
    uint64_t* fa = stage(g_a, Bn * n);
    uint64_t* fac = stage(g_acc, Bn * 2 * N);
#pragma omp parallel for
    for (size_t s = 0; s < Bn; ++s) {
        std::copy(arows[s], arows[s] + n, fa + s * n);
        for (uint32_t j = 0; j < 2; ++j) {
            NativePoly c = (*acc)[s]->GetElements()[j];
            c.SetFormat(Format::COEFFICIENT);
            const NativeVector& v = c.GetValues();
            for (uint32_t x = 0; x < N; ++x) fac[(s * 2 + j) * N + x] = v[x].ConvertToInt();
        }
    }
    check(tfhe_eval_acc(g_ctx, Bn, fa, amod, fac), "tfhe_eval_acc");
    tm.lap("device", Bn);
    std::vector<RLWECiphertext> old(Bn);
#pragma omp parallel for
    for (size_t s = 0; s < Bn; ++s) {
        std::vector<NativePoly> res(2);
        for (uint32_t j = 0; j < 2; ++j) {
            NativeVector v(N, Q);
            const uint64_t* src = fac + (s * 2 + j) * N;
            for (uint32_t x = 0; x < N; ++x) v[x] = src[x];
            res[j] = NativePoly(polyParams, Format::COEFFICIENT, false);
            res[j].SetValues(std::move(v), Format::COEFFICIENT);
        }
        old[s] = std::move((*acc)[s]);
        (*acc)[s] = std::make_shared<RLWECiphertextImpl>(std::move(res));
    }
    release_later(old);
    tm.lap("marshal out", Bn);
}

void GPUFFTBootstrap::MKMSwitch_CUDA(const std::shared_ptr<LWECryptoParams> params,
                                     std::shared_ptr<std::vector<LWECiphertext>> ctExt, NativeInteger fmod) {
    need_setup("MKMSwitch_CUDA");
    Timer tm("MKMSwitch");
    const size_t Bn = ctExt->size();
    if (Bn == 0) return;
    const uint32_t N = params->GetN(), n = params->Getn();
    // inputs stay in the extracted ciphertexts (their a rows are read in place); outputs are new
    // objects of length n mod fmod (bootstrapping.cu:1898,1926) whose rows the staging fills
    std::vector<const uint64_t*> arows(Bn);
    std::vector<uint64_t*> orows(Bn);
    uint64_t* bin = stage(g_ext, Bn);
    uint64_t* bout = stage(g_out, Bn);
    std::vector<LWECiphertext> fresh(Bn);
    int lens_ok = 1;
#pragma omp parallel for reduction(&& : lens_ok)
    for (size_t s = 0; s < Bn; ++s) {
        const LWECiphertext& ct = (*ctExt)[s];
        lens_ok = lens_ok && ct->GetA().GetLength() == N;
        arows[s] = words(ct->GetA());
        bin[s] = ct->GetB().ConvertToInt();
        fresh[s] = std::make_shared<LWECiphertextImpl>(NativeVector(n, fmod), NativeInteger(0));
        orows[s] = words(fresh[s]->GetA());
    }
    if (!lens_ok) OPENFHE_THROW(openfhe_error, "MKMSwitch_CUDA: extracted ciphertext of the wrong length");
    tm.lap("marshal in", Bn);
    check(tfhe_mkm_switch_rows(g_ctx, Bn, arows.data(), bin, fmod.ConvertToInt(), orows.data(), bout),
          "tfhe_mkm_switch_rows");
    tm.lap("device", Bn);
#pragma omp parallel for
    for (size_t s = 0; s < Bn; ++s) {
        fresh[s]->SetB(NativeInteger(bout[s]));
        std::swap((*ctExt)[s], fresh[s]);
    }
    release_later(fresh);  // the extracted inputs
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
