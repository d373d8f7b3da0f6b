// time_estimate.cpp -- the reference's GPU timing example (src/binfhe/examples/time-estimate.cpp:
// EvalBinGate, EvalFunc, EvalFloor, EvalSign, EvalDecomp on one batch each, "ms / ctx") written
// against this engine's C-ABI (include/tfhe_hip.h) from plain C++, compiled with g++ and linked
// to tfhe-gpu_amd/lib/libtfhe_hip.so -- the shape of a C++ caller that replaces the reference's
// GPUFFTBootstrap (INTEGRATION.md shows the OpenFHE-side shim).
//
// The parameter contexts are the reference example's (time-estimate.cpp:30-199): STD128 NAND;
// STD128 arbFunc logQ = 12, throw = 1 with f(x) = x^3 mod p; EvalFloor logQ = 11; EvalSign
// logQ = 17; EvalDecomp logQ = 23.  Keys and ciphertexts are synthetic (seeded splitmix64; the
// reference's KeyGen/Encrypt live in OpenFHE, outside this boundary), so outputs are not
// decrypted here -- tests/test_gpu_parity.py checks the same entry points bit for bit against
// the oracle.  Prints one line per operation and a checksum of its outputs.
//
// Usage: time_estimate [batch = 16384] [ops = gate,func,floor,sign,decomp]
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "tfhe_hip.h"

namespace {

struct SplitMix {
    uint64_t s;
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    uint64_t below(uint64_t m) { return next() % m; }
};

void check(tfhe_status s, const char* what) {
    if (s != TFHE_OK) {
        std::fprintf(stderr, "%s: %s (%s)\n", what, tfhe_status_string(s), tfhe_last_error());
        std::exit(1);
    }
}

uint64_t fnv(const std::vector<uint64_t>& v) {
    uint64_t h = 0xcbf29ce484222325ull;
    for (uint64_t x : v)
        for (int b = 0; b < 8; ++b) h = (h ^ ((x >> (8 * b)) & 0xff)) * 0x100000001b3ull;
    return h;
}

// GPUSetup with synthetic keys (the reference: KeyGen + BTKeyGen + GPUSetup)
tfhe_ctx* setup(const tfhe_params& p, SplitMix& rng) {
    const size_t bsk_words = (size_t)p.n * 2 * p.dG2 * 2 * p.N;
    const size_t ksk_words = (size_t)p.N * p.baseKS * p.dKS * (p.n + 1);
    std::vector<uint64_t> bsk(bsk_words), ksk(ksk_words);
    for (auto& x : bsk) x = rng.below(p.Q);
    for (auto& x : ksk) x = rng.below(p.qKS);
    tfhe_ctx* ctx = nullptr;
    check(tfhe_setup(&ctx, &p, bsk.data(), ksk.data(), 1), "tfhe_setup");
    return ctx;
}

std::vector<uint64_t> random_cts(const tfhe_params& p, size_t B, uint64_t mod, SplitMix& rng) {
    std::vector<uint64_t> ct(B * (p.n + 1));
    for (auto& x : ct) x = rng.below(mod);
    return ct;
}

template <typename F>
double time_ms(F&& f) {
    const auto t0 = std::chrono::high_resolution_clock::now();
    f();
    const auto t1 = std::chrono::high_resolution_clock::now();
    return std::chrono::duration<double, std::milli>(t1 - t0).count();
}

void report(const char* op, double ms, size_t B, const tfhe_ctx* ctx, const std::vector<uint64_t>& out) {
    tfhe_info info{};
    check(tfhe_get_info(const_cast<tfhe_ctx*>(ctx), &info), "tfhe_get_info");
    std::printf("%-11s batch %6zu  %8.4f ms / ctx  (%.1f ms, blind rotations so far %llu, kernel %d)  fnv %016llx\n", op,
                B, ms / (double)B, ms, (unsigned long long)info.bootstraps, info.br_kernel,
                (unsigned long long)fnv(out));
}

}  // namespace

int main(int argc, char** argv) {
    const size_t B = argc > 1 ? (size_t)std::strtoull(argv[1], nullptr, 10) : 16384;
    const std::string ops = argc > 2 ? argv[2] : "gate,func,floor,sign,decomp";
    auto want = [&](const char* op) { return ops.find(op) != std::string::npos; };
    SplitMix rng{1};
    std::printf("C-ABI version %d\n", tfhe_abi_version());

    if (want("gate")) {  // time-estimate.cpp:30-56
        tfhe_params p;
        check(tfhe_params_from_set(TFHE_STD128, &p), "params");
        tfhe_ctx* ctx = setup(p, rng);
        auto c1 = random_cts(p, B, p.q, rng), c2 = random_cts(p, B, p.q, rng);
        std::vector<uint64_t> out(B * (p.n + 1));
        check(tfhe_eval_bin_gate(ctx, TFHE_NAND, B, c1.data(), c2.data(), p.q, out.data()), "warm-up");
        const double ms = time_ms([&] { check(tfhe_eval_bin_gate(ctx, TFHE_NAND, B, c1.data(), c2.data(), p.q, out.data()), "gate"); });
        report("EvalBinGate", ms, B, ctx, out);
        check(tfhe_clean(ctx), "clean");
    }
    if (want("func")) {  // time-estimate.cpp:58-93: f(x) = x^3 mod p, p = max plaintext space (8)
        tfhe_params p;
        check(tfhe_params_from_logq(TFHE_STD128, 1, 12, 0, 0, 1, &p), "params");
        tfhe_ctx* ctx = setup(p, rng);
        const uint64_t pt = 8;
        std::vector<uint64_t> lut(p.q);
        for (uint64_t x = 0; x < p.q; ++x) {  // GenerateLUTviaFunction over [0, q): f(x * pt / q)
            const uint64_t m = x * pt / p.q;
            lut[x] = (m < pt ? m * m * m : 0) % pt;
        }
        auto ct = random_cts(p, B, p.q, rng);
        std::vector<uint64_t> out(B * (p.n + 1));
        const double ms = time_ms([&] { check(tfhe_eval_func(ctx, B, ct.data(), p.q, lut.data(), 0, out.data()), "func"); });
        report("EvalFunc", ms, B, ctx, out);
        check(tfhe_clean(ctx), "clean");
    }
    if (want("floor")) {  // time-estimate.cpp:95-122: logQ = 11, 1 bit
        tfhe_params p;
        check(tfhe_params_from_logq(TFHE_STD128, 0, 11, 0, 0, 1, &p), "params");
        tfhe_ctx* ctx = setup(p, rng);
        auto ct = random_cts(p, B, p.q, rng);
        std::vector<uint64_t> out(B * (p.n + 1));
        const double ms = time_ms([&] { check(tfhe_eval_floor(ctx, B, ct.data(), p.q, 1, out.data()), "floor"); });
        report("EvalFloor", ms, B, ctx, out);
        check(tfhe_clean(ctx), "clean");
    }
    if (want("sign")) {  // time-estimate.cpp:124-156: logQ = 17, ciphertexts mod 2^17
        tfhe_params p;
        check(tfhe_params_from_logq(TFHE_STD128, 0, 17, 0, 0, 1, &p), "params");
        tfhe_ctx* ctx = setup(p, rng);
        const uint64_t mod = 1ull << 17;
        auto ct = random_cts(p, B, mod, rng);
        std::vector<uint64_t> out(B * (p.n + 1));
        const double ms = time_ms([&] { check(tfhe_eval_sign(ctx, B, ct.data(), mod, out.data()), "sign"); });
        report("EvalSign", ms, B, ctx, out);
        check(tfhe_clean(ctx), "clean");
    }
    if (want("decomp")) {  // time-estimate.cpp:158-191: logQ = 23, ciphertexts mod 2^23
        tfhe_params p;
        check(tfhe_params_from_logq(TFHE_STD128, 0, 23, 0, 0, 1, &p), "params");
        tfhe_ctx* ctx = setup(p, rng);
        const uint64_t mod = 1ull << 23;
        auto ct = random_cts(p, B, mod, rng);
        const uint32_t max_digits = 8;
        std::vector<uint64_t> out(B * max_digits * (p.n + 1)), moduli(max_digits);
        uint32_t nd = 0;
        const double ms = time_ms([&] {
            check(tfhe_eval_decomp(ctx, B, ct.data(), mod, max_digits, out.data(), moduli.data(), &nd), "decomp");
        });
        out.resize(B * nd * (p.n + 1));
        report("EvalDecomp", ms, B, ctx, out);
        check(tfhe_clean(ctx), "clean");
    }
    return 0;
}
