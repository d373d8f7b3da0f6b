// host_math.cpp -- see host_math.hpp.
#include <atomic>
#include "host_math.hpp"

#include <cmath>
#include <cstring>
#include <unordered_map>

#include <condition_variable>
#include <functional>
#include <mutex>

namespace tfhe {

namespace {
// One job at a time over [0, n): worker w takes the w-th of T equal ranges.
struct HostPool {
    std::mutex call, m;
    std::condition_variable cv, done_cv;
    std::vector<std::thread> workers;
    unsigned T = 0;
    uint64_t gen = 0;
    unsigned pending = 0;
    size_t n = 0;
    const std::function<void(size_t, size_t)>* job = nullptr;
    HostPool() {
        T = host_threads();
        for (unsigned w = 1; w < T; ++w) workers.emplace_back([this, w] { loop(w); });
        for (auto& t : workers) t.detach();
    }
    void piece(unsigned w) {
        const size_t per = (n + T - 1) / T, lo = std::min(n, w * per), hi = std::min(n, lo + per);
        if (hi > lo) (*job)(lo, hi);
    }
    void loop(unsigned w) {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(m);
                cv.wait(lk, [&] { return gen != seen; });
                seen = gen;
            }
            piece(w);
            std::lock_guard<std::mutex> lk(m);
            if (--pending == 0) done_cv.notify_one();
        }
    }
    void run(size_t count, const std::function<void(size_t, size_t)>& fn) {
        std::lock_guard<std::mutex> one(call);
        {
            std::lock_guard<std::mutex> lk(m);
            n = count, job = &fn;
            pending = T - 1;
            ++gen;
        }
        cv.notify_all();
        piece(0);
        std::unique_lock<std::mutex> lk(m);
        done_cv.wait(lk, [&] { return pending == 0; });
    }
};

// jobs below ~1 MiB of traffic run on the calling thread
void pool_run(size_t n, size_t bytes, const std::function<void(size_t, size_t)>& fn) {
    static HostPool* pool = new HostPool();  // intentionally leaked: workers are detached
    if (pool->T <= 1 || bytes < (1u << 20)) {
        if (n) fn(0, n);
        return;
    }
    pool->run(n, fn);
}
}  // namespace

void parallel_memcpy(void* dst, const void* src, size_t bytes) {
    pool_run(bytes, bytes, [&](size_t lo, size_t hi) { std::memcpy((char*)dst + lo, (const char*)src + lo, hi - lo); });
}

uint64_t parallel_or(const uint64_t* src, size_t n) {
    std::atomic<uint64_t> acc{0};
    pool_run(n, n * 8, [&](size_t lo, size_t hi) {
        uint64_t o = 0;
        for (size_t i = lo; i < hi; ++i) o |= src[i];
        acc.fetch_or(o, std::memory_order_relaxed);
    });
    return acc.load();
}

uint64_t parallel_narrow(void* dst, const uint64_t* src, size_t n, int wb) {
    std::atomic<uint64_t> acc{0};
    pool_run(n, n * 8, [&](size_t lo, size_t hi) {
        uint64_t o = 0;
        if (wb == 2) {
            uint16_t* d = (uint16_t*)dst;
            for (size_t i = lo; i < hi; ++i) o |= src[i], d[i] = (uint16_t)src[i];
        } else {
            uint32_t* d = (uint32_t*)dst;
            for (size_t i = lo; i < hi; ++i) o |= src[i], d[i] = (uint32_t)src[i];
        }
        acc.fetch_or(o, std::memory_order_relaxed);
    });
    return acc.load();
}

void parallel_widen(uint64_t* dst, const void* src, size_t n, int wb) {
    pool_run(n, n * 8, [&](size_t lo, size_t hi) {
        if (wb == 2) {
            const uint16_t* s = (const uint16_t*)src;
            for (size_t i = lo; i < hi; ++i) dst[i] = s[i];
        } else {
            const uint32_t* s = (const uint32_t*)src;
            for (size_t i = lo; i < hi; ++i) dst[i] = s[i];
        }
    });
}

// ---- the same over row-pointer views (HostRows); flat views take the loops above ----
void parallel_memcpy_in(uint64_t* dst, const HostIn& v, size_t off, size_t n) {
    if (v.flat) return parallel_memcpy(dst, v.flat + off, n * 8);
    pool_run(n, n * 8, [&](size_t lo, size_t hi) {
        v.walk(off + lo, off + hi, [&](const uint64_t* p, size_t at, size_t len) {
            std::memcpy(dst + lo + at, p, len * 8);
        });
    });
}

uint64_t parallel_narrow_in(void* dst, const HostIn& v, size_t off, size_t n, int wb) {
    if (v.flat) return parallel_narrow(dst, v.flat + off, n, wb);
    std::atomic<uint64_t> acc{0};
    pool_run(n, n * 8, [&](size_t lo, size_t hi) {
        uint64_t o = 0;
        v.walk(off + lo, off + hi, [&](const uint64_t* p, size_t at, size_t len) {
            if (wb == 2) {
                uint16_t* d = (uint16_t*)dst + lo + at;
                for (size_t i = 0; i < len; ++i) o |= p[i], d[i] = (uint16_t)p[i];
            } else {
                uint32_t* d = (uint32_t*)dst + lo + at;
                for (size_t i = 0; i < len; ++i) o |= p[i], d[i] = (uint32_t)p[i];
            }
        });
        acc.fetch_or(o, std::memory_order_relaxed);
    });
    return acc.load();
}

void parallel_memcpy_out(const HostOut& v, size_t off, const uint64_t* src, size_t n) {
    if (v.flat) return parallel_memcpy(v.flat + off, src, n * 8);
    pool_run(n, n * 8, [&](size_t lo, size_t hi) {
        v.walk(off + lo, off + hi, [&](uint64_t* p, size_t at, size_t len) { std::memcpy(p, src + lo + at, len * 8); });
    });
}

void parallel_widen_out(const HostOut& v, size_t off, const void* src, size_t n, int wb) {
    if (v.flat) return parallel_widen(v.flat + off, src, n, wb);
    pool_run(n, n * 8, [&](size_t lo, size_t hi) {
        v.walk(off + lo, off + hi, [&](uint64_t* p, size_t at, size_t len) {
            if (wb == 2) {
                const uint16_t* s = (const uint16_t*)src + lo + at;
                for (size_t i = 0; i < len; ++i) p[i] = s[i];
            } else {
                const uint32_t* s = (const uint32_t*)src + lo + at;
                for (size_t i = 0; i < len; ++i) p[i] = s[i];
            }
        });
    });
}


uint64_t powmod(uint64_t b, uint64_t e, uint64_t m) {
    uint64_t r = 1 % m;
    b %= m;
    for (; e; e >>= 1) {
        if (e & 1) r = mulmod(r, b, m);
        b = mulmod(b, b, m);
    }
    return r;
}

bool is_prime(uint64_t x) {
    // deterministic Miller-Rabin, valid for all 64-bit x
    static const uint64_t bases[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
    if (x < 2) return false;
    for (uint64_t b : bases) {
        if (x == b) return true;
        if (x % b == 0) return false;
    }
    uint64_t d = x - 1;
    int s = 0;
    while ((d & 1) == 0) d >>= 1, ++s;
    for (uint64_t b : bases) {
        uint64_t y = powmod(b, d, x);
        if (y == 1 || y == x - 1) continue;
        bool witness = true;
        for (int r = 1; r < s && witness; ++r) {
            y = mulmod(y, y, x);
            if (y == x - 1) witness = false;
        }
        if (witness) return false;
    }
    return true;
}

uint32_t ilog2(uint64_t x) {
    uint32_t r = 0;
    while (x > 1) x >>= 1, ++r;
    return r;
}

uint32_t bitrev(uint32_t x, uint32_t bits) {
    uint32_t r = 0;
    for (uint32_t i = 0; i < bits; ++i) r = (r << 1) | ((x >> i) & 1u);
    return r;
}

// nbtheory.cpp:481-516 (FirstPrime) and :565-579 (PreviousPrime): primes = 1 mod m
static uint64_t first_prime(uint32_t bits, uint64_t m) {
    uint64_t r = powmod(2, bits, m);
    uint64_t c = (uint64_t(1) << bits) + (r ? (m - r) + 1 : 1);
    while (!is_prime(c)) c += m;
    return c;
}
static uint64_t previous_prime(uint64_t q, uint64_t m) {
    uint64_t c = q - m;
    while (!is_prime(c)) c -= m;
    return c;
}

tfhe_status params_finish(tfhe_params* p, std::string* err) {
    auto fail = [&](const char* m) {
        if (err) *err = m;
        return TFHE_ERR_INVALID_ARGUMENT;
    };
    if (p->N < 16 || (p->N & (p->N - 1))) return fail("N must be a power of two >= 16");
    if (p->baseG < 2 || (p->baseG & (p->baseG - 1))) return fail("gadget base must be a power of two");
    if (p->Q < 3 || p->Q % (2ull * p->N) != 1) return fail("Q must be a prime = 1 mod 2N");
    if (p->Q >= (1ull << 58)) return fail("Q >= 2^58 not supported");
    if (p->q == 0 || (2ull * p->N) % p->q != 0) return fail("q must divide 2N");
    if (p->qKS < 2 || p->baseKS < 2) return fail("bad key-switching modulus/base");
    // rgsw-cryptoparameters.h:87 and lwe-pke.cpp:305: natural-log ratios, as the reference computes them
    p->digitsG = (uint32_t)std::ceil(std::log((double)p->Q) / std::log((double)p->baseG));
    p->dKS = (uint32_t)std::ceil(std::log((double)p->qKS) / std::log((double)p->baseKS));
    if (p->digitsG <= p->numDigitsToThrow) return fail("numDigitsToThrow leaves no gadget digit");
    p->dG2 = 2 * (p->digitsG - p->numDigitsToThrow);
    return TFHE_OK;
}

tfhe_status params_from_set(int set, tfhe_params* p) {
    // binfhecontext.cpp:137-155 (numberBits, cyclOrder, n, q, qKS [0 = Q], baseKS, baseG)
    struct Row { int set; uint32_t bits, cycl, n, q; uint64_t qks; uint32_t bks, g; };
    static const Row rows[] = {
        {TFHE_TOY, 27, 1024, 64, 512, 0, 25, 1u << 9},
        {TFHE_MEDIUM, 28, 2048, 422, 1024, 1u << 14, 1u << 7, 1u << 10},
        {TFHE_STD128_AP, 27, 2048, 512, 1024, 1u << 14, 1u << 7, 1u << 9},
        {TFHE_STD128_APOPT, 27, 2048, 502, 1024, 1u << 14, 1u << 7, 1u << 9},
        {TFHE_STD128, 27, 2048, 512, 1024, 1u << 14, 1u << 7, 1u << 7},
        {TFHE_STD128_OPT, 27, 2048, 502, 1024, 1u << 14, 1u << 7, 1u << 7},
        {TFHE_STD192, 37, 4096, 1024, 1024, 1u << 19, 28, 1u << 14},
        {TFHE_STD192_OPT, 37, 4096, 805, 1024, 1u << 15, 32, 1u << 13},
        {TFHE_STD256, 29, 4096, 1024, 2048, 1u << 14, 1u << 7, 1u << 8},
        {TFHE_STD256_OPT, 29, 4096, 990, 2048, 1u << 14, 1u << 7, 1u << 8},
        {TFHE_STD128Q, 50, 4096, 1024, 1024, 1u << 25, 32, 1u << 25},
        {TFHE_STD128Q_OPT, 50, 4096, 585, 1024, 1u << 15, 32, 1u << 25},
        {TFHE_STD192Q, 35, 4096, 1024, 1024, 1u << 17, 64, 1u << 14},
        {TFHE_STD192Q_OPT, 35, 4096, 875, 1024, 1u << 15, 32, 1u << 12},
        {TFHE_STD256Q, 27, 4096, 2048, 2048, 1u << 16, 16, 1u << 7},
        {TFHE_STD256Q_OPT, 27, 4096, 1225, 1024, 1u << 16, 16, 1u << 7},
        {TFHE_SIGNED_MOD_TEST, 28, 2048, 512, 1024, 0, 25, 1u << 7},
    };
    for (const Row& r : rows) {
        if (r.set != set) continue;
        std::memset(p, 0, sizeof(*p));
        p->Q = previous_prime(first_prime(r.bits, r.cycl), r.cycl);
        p->N = r.cycl / 2;
        p->n = r.n;
        p->q = r.q;
        p->qKS = r.qks ? r.qks : p->Q;
        p->baseKS = r.bks;
        p->baseG = r.g;
        return params_finish(p, nullptr);
    }
    return TFHE_ERR_INVALID_ARGUMENT;
}

// StdLatticeParm::FindRingDim(HEStd_ternary, HEStd_128_classic, logQ), stdlatticeparms.cpp:110-130
static uint32_t ring_dim_ternary128(uint32_t logQ) {
    static const uint32_t dim[] = {1024, 2048, 4096, 8192, 16384, 32768, 65536};
    static const uint32_t maxlogq[] = {27, 54, 109, 218, 438, 881, 1772};
    uint32_t prev = 0;
    for (int i = 0; i < 7; ++i) {
        if (logQ <= maxlogq[i] && logQ > prev) return dim[i];
        prev = maxlogq[i];
    }
    return 131072;
}

tfhe_status params_from_logq(int set, int arb_func, uint32_t logQ, int64_t N, uint32_t baseG, uint32_t thr,
                             tfhe_params* p) {
    // binfhecontext.cpp:51-113
    if (set != TFHE_STD128 && set != TFHE_TOY) return TFHE_ERR_UNSUPPORTED;
    if (logQ > 29 || logQ < 11) return TFHE_ERR_UNSUPPORTED;
    uint32_t logQprime = 54;
    if (baseG == 0) {
        if (logQ > 25) baseG = 1u << 14;
        else if (logQ > 16) baseG = 1u << 18;
        else if (logQ > 11) baseG = 1u << 27;
        else baseG = 1u << 5, logQprime = 27;
    }
    uint32_t ring = ring_dim_ternary128(logQprime);
    if (N >= (int64_t)ring) ring = (uint32_t)N;
    std::memset(p, 0, sizeof(*p));
    p->Q = previous_prime(first_prime(logQprime, 2ull * ring), 2ull * ring);
    p->N = ring;
    p->q = arb_func ? ring : 2ull * ring;
    p->qKS = 1ull << 35;
    p->n = set == TFHE_TOY ? 32 : 1305;
    p->baseKS = 32;
    p->baseG = baseG;
    p->numDigitsToThrow = thr;
    return params_finish(p, nullptr);
}

int word_bits_for(const tfhe_params& p) {
    if (p.Q < (1ull << 31) && (u128)2 * p.dG2 * p.Q < ((u128)1 << 32)) return 32;
    return 64;
}

NttTables make_ntt_tables(uint64_t Q, uint32_t N) {
    NttTables t;
    t.N = N;
    t.logN = ilog2(N);
    t.Q = Q;
    // psi = RootOfUnity(2N, Q) as OpenFHE picks it (rgsw-cryptoparameters.h:80,
    // nbtheory.cpp:284-343): the smallest primitive 2N-th root, i.e. the minimum over the
    // odd powers of any one of them.  With OpenFHE's bit-reversed table and transform
    // (transformnat-impl.h:196-236, 684-706) the NTT below then IS OpenFHE's EVALUATION
    // format, so evaluation-format keys need no conversion (tfhe_setup_eval).
    uint64_t r = 0;
    for (uint64_t g = 2;; ++g) {
        r = powmod(g, (Q - 1) / (2ull * N), Q);
        if (powmod(r, N, Q) == Q - 1) break;
    }
    t.psi = r;
    const uint64_t r2 = mulmod(r, r, Q);
    for (uint64_t k = 3, x = r; k < 2ull * N; k += 2) {
        x = mulmod(x, r2, Q);
        if (x < t.psi) t.psi = x;
    }
    uint64_t ipsi = powmod(t.psi, Q - 2, Q);
    t.Ninv = powmod(N, Q - 2, Q);
    t.psi_br.resize(N);
    t.ipsi_br.resize(N);
    for (uint32_t k = 0; k < N; ++k) {
        uint32_t e = bitrev(k, t.logN);
        t.psi_br[k] = powmod(t.psi, e, Q);
        t.ipsi_br[k] = powmod(ipsi, e, Q);
    }
    t.mono.resize(2ull * N);
    std::unordered_map<uint64_t, uint32_t> dlog;
    uint64_t pw = 1;
    for (uint32_t k = 0; k < 2 * N; ++k) {
        t.mono[k] = submod(pw, 1, Q);
        dlog[pw] = k;
        pw = mulmod(pw, t.psi, Q);
    }
    // e_x from the transform itself: NTT(X)[x] = psi^(e_x)
    std::vector<uint64_t> x(N, 0);
    x[1] = 1;
    host_ntt_fwd(t, x.data());
    t.eidx.resize(N);
    for (uint32_t k = 0; k < N; ++k) t.eidx[k] = dlog.at(x[k]);
    return t;
}

void host_ntt_fwd(const NttTables& t, uint64_t* a) {
    const uint64_t Q = t.Q;
    uint32_t len = t.N;
    for (uint32_t m = 1; m < t.N; m <<= 1) {
        len >>= 1;
        for (uint32_t i = 0; i < m; ++i) {
            const uint64_t S = t.psi_br[m + i];
            for (uint32_t j = 2 * i * len; j < 2 * i * len + len; ++j) {
                uint64_t U = a[j], V = mulmod(a[j + len], S, Q);
                a[j] = addmod(U, V, Q);
                a[j + len] = submod(U, V, Q);
            }
        }
    }
}

void host_ntt_inv(const NttTables& t, uint64_t* a, bool scale) {
    const uint64_t Q = t.Q;
    uint32_t len = 1;
    for (uint32_t m = t.N; m > 1; m >>= 1, len <<= 1) {
        const uint32_t h = m >> 1;
        for (uint32_t i = 0; i < h; ++i) {
            const uint64_t S = t.ipsi_br[h + i];
            for (uint32_t j = 2 * i * len; j < 2 * i * len + len; ++j) {
                uint64_t U = a[j], V = a[j + len];
                a[j] = addmod(U, V, Q);
                a[j + len] = mulmod(submod(U, V, Q), S, Q);
            }
        }
    }
    if (scale)
        for (uint32_t j = 0; j < t.N; ++j) a[j] = mulmod(a[j], t.Ninv, Q);
}

bool bsk_to_ntt_scaled(const tfhe_params& p, const NttTables& t, const uint64_t* bsk, bool eval, uint64_t* out) {
    const size_t polys = (size_t)p.n * 2 * p.dG2 * 2;
    const uint32_t N = p.N;
    std::atomic<bool> bad{false};
    parallel_for(polys, [&](size_t k) {
        uint64_t* dst = out + (size_t)k * N;
        const uint64_t* src = bsk + (size_t)k * N;
        if (eval) {  // already OpenFHE's NTT: entries must be reduced (NativePoly values)
            for (uint32_t x = 0; x < N; ++x) {
                if (src[x] >= p.Q) bad = true;
                dst[x] = mulmod(src[x] % p.Q, t.Ninv, p.Q);
            }
            return;
        }
        for (uint32_t x = 0; x < N; ++x) dst[x] = src[x] % p.Q;
        host_ntt_fwd(t, dst);
        for (uint32_t x = 0; x < N; ++x) dst[x] = mulmod(dst[x], t.Ninv, p.Q);
    });
    return !bad;
}

}  // namespace tfhe
