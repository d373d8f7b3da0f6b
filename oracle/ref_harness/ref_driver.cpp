// ref_driver.cpp -- TEST INFRASTRUCTURE (oracle/_ref only; never shipped).
//
// Drives the REFERENCE's own OpenFHE BinFHE code (compiled from /root/reference by
// oracle/Makefile.ref) on seeded inputs, so its outputs can be committed as golden
// vectors (tools/gen_golden.py) and compared with the MI355X engine.  Two binaries share
// this file:
//   ref_kat    + cpu_boundary.cpp : the 7 GPU symbols served by the reference's CPU functions
//   ref_dropin + tfhe-gpu_amd/shim/bootstrapping_hip.cpp : the 7 symbols served by the HIP
//              engine through its C-ABI -- the reference's vector code, unchanged, on MI355X.
//
// Usage: ref_driver key=value ...
//   ctx=set:STD128 | ctx=logq:<SET>,<arbFunc>,<logQ>,<N>,<baseG>,<throw>
//        GenerateBinFHEContext(set, GINX) (binfhecontext.cpp:115-181) or
//        GenerateBinFHEContext(set, arbFunc, logQ, N, GINX, false, baseG, throw) (:51-113)
//   keys=synth:<seed>  SURVEY.md Appendix B: splitmix64 coefficients, SetFormat(EVALUATION),
//                      BTKeyLoad (binfhecontext.h:208-210)
//   keys=valid:<seed>  the C oracle's deterministic valid keys (or_keygen), same load path
//   op=params | lut_cube | kat | bskeval | acc | mkm | <gate> | func | funcvec | floor | sign | decomp |
//      mulmatrix (CiphertextMulMatrix, binfhecontext.cpp:319-321: in = ciphertexts mod `mod`, matrix =
//      int64 [K][cols] file, cols=<cols>, modulus=<m>; impl=cpugemm: the reference's own CPU function
//      CPUGEMM, examples/GEMM.cpp:30-56, compiled from that file (its main renamed) instead)
//   api=vector (default; through the 7 boundary symbols) | single (CPU single-ciphertext API)
//   in=<u64 file> in2=<u64 file> lut=<u64 file> acc=<u64 file> mod=<ct modulus> fmod=<m>
//   roundbits=<r> out=<u64 file> gpus=<numGPUs for GPUSetup> reps=<timed repetitions>
//   sizes=<B1,B2,...>  batch sweep (gates / func / floor / sign / decomp): the reps are timed on the
//                      first B1, then B2, ... ciphertexts of the input, keys loaded once (the
//                      reference's CHES-experiments.cpp:95-121 sweep); "sweep" lists best/mean per size
//   batch=<file>       several ops on one context and key load: one line of key=value overrides per op
// Prints one JSON line (digests, timings) on stdout (one per op in batch mode).
#include "binfhecontext.h"
#include "rgsw-acc-cggi.h"
#include "bootstrapping.cuh"
#include "tfhe_oracle.h"

// the reference's CPU CiphertextMulMatrix check (examples/GEMM.cpp:30-56; Makefile.ref compiles that file
// with its main renamed)
std::vector<lbcrypto::LWECiphertext> CPUGEMM(lbcrypto::BinFHEContext cc, std::vector<lbcrypto::LWECiphertext> ct_vec,
                                             std::vector<std::vector<int64_t>> matrix);

#include <omp.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

using namespace lbcrypto;

namespace {

std::map<std::string, std::string> g_args;

std::string arg(const std::string& k, const std::string& dflt = "") {
    auto it = g_args.find(k);
    return it == g_args.end() ? dflt : it->second;
}
uint64_t arg_u64(const std::string& k, uint64_t dflt = 0) {
    auto s = arg(k);
    return s.empty() ? dflt : std::stoull(s);
}

[[noreturn]] void die(const std::string& msg) {
    fprintf(stderr, "ref_driver: %s\n", msg.c_str());
    exit(2);
}

const char* kSets[] = {"TOY", "MEDIUM", "STD128_AP", "STD128_APOPT", "STD128", "STD128_OPT",
                       "STD192", "STD192_OPT", "STD256", "STD256_OPT", "STD128Q", "STD128Q_OPT",
                       "STD192Q", "STD192Q_OPT", "STD256Q", "STD256Q_OPT", "SIGNED_MOD_TEST"};
int set_id(const std::string& s) {
    for (int i = 0; i < (int)(sizeof(kSets) / sizeof(kSets[0])); ++i)
        if (s == kSets[i]) return i;
    die("unknown parameter set " + s);
}

std::vector<std::string> split(const std::string& s, char c) {
    std::vector<std::string> r;
    std::stringstream ss(s);
    std::string t;
    while (std::getline(ss, t, c)) r.push_back(t);
    return r;
}

std::vector<uint64_t> read_u64(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) die("cannot read " + path);
    f.seekg(0, std::ios::end);
    size_t bytes = f.tellg();
    f.seekg(0);
    std::vector<uint64_t> v(bytes / 8);
    f.read(reinterpret_cast<char*>(v.data()), bytes);
    return v;
}
void write_u64(const std::string& path, const std::vector<uint64_t>& v) {
    if (path.empty()) return;
    std::ofstream f(path, std::ios::binary);
    f.write(reinterpret_cast<const char*>(v.data()), v.size() * 8);
}

uint64_t fnv1a64(const uint64_t* w, size_t count, uint64_t h = 0xcbf29ce484222325ULL) {
    for (size_t i = 0; i < count; ++i)
        for (int b = 0; b < 8; ++b) {
            h ^= (w[i] >> (8 * b)) & 0xff;
            h *= 0x100000001b3ULL;
        }
    return h;
}
std::string hex64(uint64_t h) {
    char buf[17];
    snprintf(buf, sizeof buf, "%016llx", (unsigned long long)h);
    return buf;
}

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ---- context, keys ----------------------------------------------------------------------
struct Setup {
    BinFHEContext cc;
    or_params op{};
    uint32_t n = 0, N = 0, dG2 = 0, baseKS = 0, dKS = 0;
    NativeInteger q, Q, qKS;
};

void make_context(Setup& s) {
    auto spec = arg("ctx", "set:STD128");
    if (spec.rfind("set:", 0) == 0) {
        int id = set_id(spec.substr(4));
        s.cc.GenerateBinFHEContext(static_cast<BINFHE_PARAMSET>(id), GINX);
        if (or_params_from_set(id, &s.op)) die("oracle has no params for " + spec);
    } else if (spec.rfind("logq:", 0) == 0) {
        auto f = split(spec.substr(5), ',');
        if (f.size() != 6) die("ctx=logq:<SET>,<arb>,<logQ>,<N>,<baseG>,<throw>");
        int id = set_id(f[0]);
        bool arb = std::stoi(f[1]) != 0;
        uint32_t logQ = std::stoul(f[2]), baseG = std::stoul(f[4]), thr = std::stoul(f[5]);
        int64_t N = std::stoll(f[3]);
        s.cc.GenerateBinFHEContext(static_cast<BINFHE_PARAMSET>(id), arb, logQ, N, GINX, false, baseG, thr);
        if (or_params_from_logq(id, arb, logQ, N, baseG, thr, &s.op)) die("oracle has no params for " + spec);
    } else {
        die("bad ctx " + spec);
    }
    auto L = s.cc.GetParams()->GetLWEParams();
    auto R = s.cc.GetParams()->GetRingGSWParams();
    s.n = L->Getn();
    s.N = L->GetN();
    s.q = L->Getq();
    s.Q = L->GetQ();
    s.qKS = L->GetqKS();
    s.baseKS = L->GetBaseKS();
    s.dG2 = 2 * (R->GetDigitsG() - R->GetNumDigitsToThrow());
    s.dKS = (uint32_t)std::ceil(std::log(s.qKS.ConvertToDouble()) / std::log((double)s.baseKS));
    if (s.op.n != s.n || s.op.N != s.N || s.op.Q != s.Q.ConvertToInt() || s.op.dG2 != s.dG2 || s.op.dKS != s.dKS)
        die("oracle parameter record disagrees with the reference context");
}

// Loads [n][2][dG2][2][N] coefficient-form words (and KSK [N][baseKS][dKS][n+1]) as
// OpenFHE keys: each polynomial SetFormat(EVALUATION), as KeyGenAcc leaves them.
void load_keys(Setup& s, const uint64_t* bsk_coeff, const uint64_t* ksk) {
    auto R = s.cc.GetParams()->GetRingGSWParams();
    auto polyParams = R->GetPolyParams();
    const uint32_t n = s.n, N = s.N, dG2 = s.dG2;
    auto acc = std::make_shared<RingGSWACCKeyImpl>(1, 2, n);
#pragma omp parallel for collapse(2)
    for (uint32_t i = 0; i < n; ++i)
        for (uint32_t key = 0; key < 2; ++key) {
            std::vector<std::vector<NativePoly>> el(dG2, std::vector<NativePoly>(2));
            for (uint32_t l = 0; l < dG2; ++l)
                for (uint32_t m = 0; m < 2; ++m) {
                    NativeVector v(N, s.Q);
                    const uint64_t* src = bsk_coeff + ((((size_t)i * 2 + key) * dG2 + l) * 2 + m) * N;
                    for (uint32_t j = 0; j < N; ++j) v[j] = src[j];
                    NativePoly p(polyParams, Format::COEFFICIENT, false);
                    p.SetValues(std::move(v), Format::COEFFICIENT);
                    p.SetFormat(Format::EVALUATION);
                    el[l][m] = std::move(p);
                }
            (*acc)[0][key][i] = std::make_shared<RingGSWEvalKeyImpl>(el);
        }
    std::vector<std::vector<std::vector<NativeVector>>> A(
        N, std::vector<std::vector<NativeVector>>(s.baseKS, std::vector<NativeVector>(s.dKS)));
    std::vector<std::vector<std::vector<NativeInteger>>> Bk(
        N, std::vector<std::vector<NativeInteger>>(s.baseKS, std::vector<NativeInteger>(s.dKS)));
#pragma omp parallel for
    for (uint32_t i = 0; i < N; ++i)
        for (uint32_t j = 0; j < s.baseKS; ++j)
            for (uint32_t k = 0; k < s.dKS; ++k) {
                const uint64_t* row = ksk + (((size_t)i * s.baseKS + j) * s.dKS + k) * (n + 1);
                NativeVector v(n, s.qKS);
                for (uint32_t l = 0; l < n; ++l) v[l] = row[l];
                A[i][j][k] = std::move(v);
                Bk[i][j][k] = row[n];
            }
    RingGSWBTKey bt;
    bt.BSkey = acc;
    bt.KSkey = std::make_shared<LWESwitchingKeyImpl>(A, Bk);
    s.cc.BTKeyLoad(bt);
    s.cc.BTKeyMapLoadSingleElement(R->GetBaseG(), bt);  // single EvalSign/EvalDecomp read the map
}

// ---- ciphertexts ------------------------------------------------------------------------
size_t g_limit = 0;  // sizes= sweep: ciphertexts read from each input (0 = all)
bool g_batch = false;      // batch= mode: several ops per process
bool g_gpu_setup = false;  // batch= mode: GPUSetup done (by the first vector op, again when gpus= changes)
int g_gpus = 0;

std::vector<LWECiphertext> read_cts(const std::string& path, uint32_t n, uint64_t mod) {
    auto w = read_u64(path);
    if (w.size() % (n + 1)) die(path + ": size is not a multiple of n+1");
    std::vector<LWECiphertext> v(w.size() / (n + 1));
    if (g_limit) {
        if (g_limit > v.size()) die(path + ": fewer ciphertexts than the sweep size");
        v.resize(g_limit);
    }
    for (size_t s = 0; s < v.size(); ++s) {
        NativeVector a(n, mod);
        for (uint32_t l = 0; l < n; ++l) a[l] = w[s * (n + 1) + l];
        v[s] = std::make_shared<LWECiphertextImpl>(std::move(a), NativeInteger(w[s * (n + 1) + n]));
    }
    return v;
}
void append_ct(std::vector<uint64_t>& out, const LWECiphertext& c) {
    const auto& a = c->GetA();
    for (size_t l = 0; l < a.GetLength(); ++l) out.push_back(a[l].ConvertToInt());
    out.push_back(c->GetB().ConvertToInt());
}

NativeInteger cube_mod(NativeInteger m, NativeInteger p1) {  // time-estimate.cpp:69-74
    if (m < p1)
        return (m * m * m) % p1;
    return ((m - p1 / 2) * (m - p1 / 2) * (m - p1 / 2)) % p1;
}

BINGATE gate_of(const std::string& g) {
    static const std::map<std::string, BINGATE> m = {{"OR", OR},     {"AND", AND},   {"NOR", NOR},
                                                    {"NAND", NAND}, {"XOR", XOR},   {"XNOR", XNOR},
                                                    {"XOR_FAST", XOR_FAST}, {"XNOR_FAST", XNOR_FAST}};
    auto it = m.find(g);
    if (it == m.end()) die("unknown op " + g);
    return it->second;
}

}  // namespace

int run_op(Setup& s, or_rng& rng, std::ostringstream& js);

int main(int argc, char** argv) {
    for (int i = 1; i < argc; ++i) {
        const char* e = strchr(argv[i], '=');
        if (!e) die(std::string("argument without '=': ") + argv[i]);
        g_args[std::string(argv[i], e - argv[i])] = e + 1;
    }
    const std::string op = arg("op");
    Setup s;
    make_context(s);
    std::ostringstream js;
    js << "{\"op\":\"" << op << "\"";

    if (op == "params") {
        auto R = s.cc.GetParams()->GetRingGSWParams();
        js << ",\"n\":" << s.n << ",\"N\":" << s.N << ",\"q\":" << s.q.ConvertToInt() << ",\"Q\":"
           << s.Q.ConvertToInt() << ",\"baseG\":" << R->GetBaseG() << ",\"dG2\":" << s.dG2
           << ",\"qKS\":" << s.qKS.ConvertToInt() << ",\"baseKS\":" << s.baseKS << ",\"dKS\":" << s.dKS
           << ",\"numDigitsToThrow\":" << R->GetNumDigitsToThrow() << ",\"maxPlaintext\":"
           << s.cc.GetMaxPlaintextSpace().ConvertToInt() << ",\"gateConst\":[";
        for (size_t g = 0; g < R->GetGateConst().size(); ++g)
            js << (g ? "," : "") << R->GetGateConst()[g].ConvertToInt();
        js << "]}";
        printf("%s\n", js.str().c_str());
        return 0;
    }
    if (op == "lut_cube") {  // GenerateLUTviaFunction(x^3 mod p, p) (binfhecontext.cpp:280-301)
        uint64_t p = arg_u64("p", s.cc.GetMaxPlaintextSpace().ConvertToInt());
        auto lut = s.cc.GenerateLUTviaFunction(cube_mod, NativeInteger(p));
        std::vector<uint64_t> w;
        for (auto& x : lut) w.push_back(x.ConvertToInt());
        write_u64(arg("out"), w);
        js << ",\"p\":" << p << ",\"len\":" << w.size() << ",\"fnv\":\"" << hex64(fnv1a64(w.data(), w.size()))
           << "\"}";
        printf("%s\n", js.str().c_str());
        return 0;
    }

    // keys
    const auto keys = arg("keys", "synth:1");
    const uint64_t seed = std::stoull(keys.substr(keys.find(':') + 1));
    or_rng rng{seed};
    double t0 = now_s();
    {
        std::vector<uint64_t> bsk((size_t)s.n * 2 * s.dG2 * 2 * s.N);
        std::vector<uint64_t> ksk((size_t)s.N * s.baseKS * s.dKS * (s.n + 1));
        if (keys.rfind("synth:", 0) == 0) {
            or_kat_keys(&s.op, &rng, bsk.data(), ksk.data());  // SURVEY Appendix B order
        } else if (keys.rfind("valid:", 0) == 0) {
            std::vector<uint64_t> sk(s.n);
            or_keygen(&s.op, &rng, sk.data(), bsk.data(), ksk.data());
        } else {
            die("bad keys " + keys);
        }
        load_keys(s, bsk.data(), ksk.data());
    }
    double t_keys = now_s() - t0;
    js << ",\"keys\":\"" << keys << "\",\"key_load_s\":" << t_keys;
    const std::string batch = arg("batch");
    if (batch.empty()) return run_op(s, rng, js);
    // batch=<file>: one op per line (key=value overrides of this command line's arguments; ctx and keys are
    // the command line's), all on the context and keys loaded above -- one JSON line per op.  Vector ops share
    // one GPUSetup, cleaned after the last (the GPU test suite's drop-in cases, tests/test_gpu_dropin.py)
    const auto base = g_args;
    std::ifstream in(batch);
    if (!in) die("cannot read " + batch);
    std::string line;
    g_batch = true;
    while (std::getline(in, line)) {
        if (line.empty()) continue;
        g_args = base;
        std::istringstream ls(line);
        std::string tok;
        while (ls >> tok) {
            const size_t e = tok.find('=');
            if (e == std::string::npos) die("batch line token without '=': " + tok);
            if (tok.compare(0, e, "ctx") == 0 || tok.compare(0, e, "keys") == 0) die("batch lines cannot change ctx / keys");
            g_args[tok.substr(0, e)] = tok.substr(e + 1);
        }
        g_limit = 0;
        std::ostringstream jl;
        jl << "{\"op\":\"" << arg("op") << "\",\"keys\":\"" << keys << "\",\"key_load_s\":" << t_keys;
        if (int r = run_op(s, rng, jl)) return r;
        fflush(stdout);
    }
    if (g_gpu_setup) s.cc.GPUClean();
    return 0;
}

int run_op(Setup& s, or_rng& rng, std::ostringstream& js) {
    const std::string op = arg("op");
    if (op == "bskeval") {  // OpenFHE's EVALUATION-format BSK, [n][2][dG2][2][N] order
        auto bt = s.cc.GetRefreshKey();
        uint64_t h = 0xcbf29ce484222325ULL;
        std::vector<uint64_t> head;
        for (uint32_t i = 0; i < s.n; ++i)
            for (uint32_t key = 0; key < 2; ++key)
                for (uint32_t l = 0; l < s.dG2; ++l)
                    for (uint32_t m = 0; m < 2; ++m) {
                        const NativePoly& p = (*(*bt)[0][key][i])[l][m];
                        if (p.GetFormat() != Format::EVALUATION) die("BSK polynomial not in EVALUATION format");
                        std::vector<uint64_t> w(s.N);
                        for (uint32_t j = 0; j < s.N; ++j) w[j] = p[j].ConvertToInt();
                        h = fnv1a64(w.data(), w.size(), h);
                        if (head.size() < 2 * s.N) head.insert(head.end(), w.begin(), w.end());
                    }
        write_u64(arg("out"), head);  // first two polynomials in full
        js << ",\"fnv\":\"" << hex64(h) << "\"}";
        printf("%s\n", js.str().c_str());
        return 0;
    }

    if (op == "kat") {  // SURVEY Appendix B trials, single-ciphertext API
        js << ",\"trials\":[";
        for (int t = 0; t < 3; ++t) {
            std::vector<uint64_t> w[2];
            NativeVector a[2] = {NativeVector(s.n, s.q), NativeVector(s.n, s.q)};
            uint64_t b[2];
            for (int c = 0; c < 2; ++c) {
                for (uint32_t l = 0; l < s.n; ++l) a[c][l] = or_splitmix64(&rng) % s.q.ConvertToInt();
                b[c] = or_splitmix64(&rng) % s.q.ConvertToInt();
            }
            auto c1 = std::make_shared<LWECiphertextImpl>(a[0], NativeInteger(b[0]));
            auto c2 = std::make_shared<LWECiphertextImpl>(a[1], NativeInteger(b[1]));
            LWECiphertext r;
            if (arg("kat", "nand") == "cube") {
                auto lut = s.cc.GenerateLUTviaFunction(cube_mod, s.cc.GetMaxPlaintextSpace());
                r = s.cc.EvalFunc(c1, lut);
            } else {
                r = s.cc.EvalBinGate(NAND, c1, c2);
            }
            std::vector<uint64_t> o;
            append_ct(o, r);
            js << (t ? "," : "") << "{\"a0_3\":[" << o[0] << "," << o[1] << "," << o[2] << "," << o[3]
               << "],\"b\":" << o.back() << ",\"mod\":" << r->GetModulus().ConvertToInt() << ",\"fnv\":\""
               << hex64(fnv1a64(o.data(), o.size())) << "\"}";
        }
        js << "]}";
        printf("%s\n", js.str().c_str());
        return 0;
    }

    const std::string api = arg("api", "vector");
    const int reps = (int)arg_u64("reps", 1);
    const int gpus = (int)arg_u64("gpus", 0);
    if (api == "vector" && (!g_gpu_setup || gpus != g_gpus)) {  // (a batch line with another gpus= sets up again)
        if (g_gpu_setup) s.cc.GPUClean();
        double ts = now_s();
        s.cc.GPUSetup(gpus);
        js << ",\"gpu_setup_s\":" << (now_s() - ts);
        g_gpu_setup = g_batch;  // a batch keeps it for its later ops
        g_gpus = gpus;
    }
    std::vector<uint64_t> out;
    double best = 1e30, total = 0;
    uint64_t extra = 0;  // decomp: digits
    std::vector<size_t> sizes;
    for (auto& f : split(arg("sizes"), ',')) sizes.push_back(std::stoull(f));
    if (sizes.empty()) sizes.push_back(0);
    // threads=<T1,T2,...> beside sizes=: the OpenMP threads of each size's runs (the reference's CPU
    // accumulator parallelises over ciphertexts), e.g. a 1-thread sample and the full one after one key load
    std::vector<int> nthreads;
    for (auto& f : split(arg("threads"), ',')) nthreads.push_back(std::stoi(f));
    if (!nthreads.empty() && nthreads.size() != sizes.size()) die("threads= needs one entry per sizes= entry");
    std::ostringstream sweep;
    for (size_t si = 0; si < sizes.size(); ++si) {
    g_limit = sizes[si];
    if (!nthreads.empty()) omp_set_num_threads(nthreads[si]);
    best = 1e30, total = 0;
    for (int rep = 0; rep < reps; ++rep) {
        out.clear();
        double ts = now_s();
        if (op == "acc") {  // boundary: EvalAcc_CUDA directly
            const uint64_t amod = arg_u64("mod");
            auto aw = read_u64(arg("in"));
            auto accw = read_u64(arg("acc"));
            const size_t B = aw.size() / s.n;
            if (accw.size() != B * 2 * s.N) die("acc file size");
            auto R = s.cc.GetParams()->GetRingGSWParams();
            std::vector<NativeVector> a(B);
            auto acc = std::make_shared<std::vector<RLWECiphertext>>(B);
            for (size_t c = 0; c < B; ++c) {
                a[c] = NativeVector(s.n, amod);
                for (uint32_t l = 0; l < s.n; ++l) a[c][l] = aw[c * s.n + l];
                std::vector<NativePoly> e(2);
                for (int j = 0; j < 2; ++j) {
                    NativeVector v(s.N, s.Q);
                    for (uint32_t x = 0; x < s.N; ++x) v[x] = accw[(c * 2 + j) * s.N + x];
                    e[j] = NativePoly(R->GetPolyParams(), Format::COEFFICIENT, false);
                    e[j].SetValues(std::move(v), Format::COEFFICIENT);
                }
                (*acc)[c] = std::make_shared<RLWECiphertextImpl>(std::move(e));
            }
            ts = now_s();
            if (api == "vector") {
                GPUFFTBootstrap::EvalAcc_CUDA(R, a, acc, 0);
            } else {  // single: the CPU accumulator + transpose, as rgsw-acc-cggi.cpp / BootstrapGateCore use it
                RingGSWAccumulatorCGGI accum;
                for (size_t c = 0; c < B; ++c) {
                    auto e = (*acc)[c]->GetElements();
                    e[0].SetFormat(Format::EVALUATION);
                    e[1].SetFormat(Format::EVALUATION);
                    auto rc = std::make_shared<RLWECiphertextImpl>(std::move(e));
                    accum.EvalAcc(R, s.cc.GetRefreshKey(), rc, a[c], "NTT", 0);
                    auto r = rc->GetElements();
                    r[0] = r[0].Transpose();
                    r[0].SetFormat(Format::COEFFICIENT);
                    r[1].SetFormat(Format::COEFFICIENT);
                    (*acc)[c] = std::make_shared<RLWECiphertextImpl>(std::move(r));
                }
            }
            double dt = now_s() - ts;
            best = std::min(best, dt);
            total += dt;
            for (size_t c = 0; c < B; ++c)
                for (int j = 0; j < 2; ++j) {
                    const auto& p = (*acc)[c]->GetElements()[j];
                    for (uint32_t x = 0; x < s.N; ++x) out.push_back(p[x].ConvertToInt());
                }
            continue;
        }
        if (op == "mkm") {  // boundary: MKMSwitch_CUDA directly
            auto w = read_u64(arg("in"));
            const size_t B = w.size() / (s.N + 1);
            auto ext = std::make_shared<std::vector<LWECiphertext>>(B);
            for (size_t c = 0; c < B; ++c) {
                NativeVector a(s.N, s.Q);
                for (uint32_t l = 0; l < s.N; ++l) a[l] = w[c * (s.N + 1) + l];
                (*ext)[c] = std::make_shared<LWECiphertextImpl>(std::move(a), NativeInteger(w[c * (s.N + 1) + s.N]));
            }
            ts = now_s();
            NativeInteger fmod(arg_u64("fmod"));
            if (api == "vector") {
                GPUFFTBootstrap::MKMSwitch_CUDA(s.cc.GetParams()->GetLWEParams(), ext, fmod);
            } else {
                LWEEncryptionScheme lwe;
                auto L = s.cc.GetParams()->GetLWEParams();
                for (auto& c : *ext) c = lwe.ModSwitch(fmod, lwe.KeySwitch(L, s.cc.GetSwitchKey(), lwe.ModSwitch(L->GetqKS(), c)));
            }
            double dt = now_s() - ts;
            best = std::min(best, dt);
            total += dt;
            for (auto& c : *ext) append_ct(out, c);
            continue;
        }

        if (op == "mulmatrix") {  // vector API only (no single-ciphertext counterpart)
            auto ct = read_cts(arg("in"), s.n, arg_u64("mod", s.q.ConvertToInt()));
            auto mw = read_u64(arg("matrix"));
            const size_t cols = arg_u64("cols");
            if (cols == 0 || mw.size() != ct.size() * cols) die("matrix file must hold [K][cols] int64");
            std::vector<std::vector<int64_t>> m(ct.size(), std::vector<int64_t>(cols));
            for (size_t k = 0; k < ct.size(); ++k)
                for (size_t c = 0; c < cols; ++c) m[k][c] = (int64_t)mw[k * cols + c];
            ts = now_s();
            // impl=cpugemm: GEMM.cpp's CPUGEMM, which takes the context's qKS as the modulus
            if (arg("impl", "") == "cpugemm" && arg_u64("modulus") != s.cc.GetParams()->GetLWEParams()->GetqKS().ConvertToInt())
                die("impl=cpugemm reduces mod the context's qKS: modulus must equal it");
            auto res = arg("impl", "") == "cpugemm" ? CPUGEMM(s.cc, ct, m) : s.cc.CiphertextMulMatrix(ct, m, arg_u64("modulus"));
            double dt = now_s() - ts;
            best = std::min(best, dt);
            total += dt;
            for (auto& c : res) append_ct(out, c);
            continue;
        }
        const uint64_t mod = arg_u64("mod", s.q.ConvertToInt());
        auto ct = read_cts(arg("in"), s.n, mod);
        std::vector<LWECiphertext> res;
        std::vector<std::vector<LWECiphertext>> dres;
        ts = now_s();
        if (op == "func" || op == "funcvec") {
            auto lw = read_u64(arg("lut"));
            if (op == "func") {
                std::vector<NativeInteger> lut(lw.begin(), lw.end());
                if (api == "vector") {
                    res = s.cc.EvalFunc(ct, lut);
                } else {
                    for (auto& c : ct) res.push_back(s.cc.EvalFunc(c, lut));
                }
            } else {
                if (lw.size() != ct.size() * mod) die("funcvec: lut must be [B][mod]");
                std::vector<std::vector<NativeInteger>> luts(ct.size());
                for (size_t c = 0; c < ct.size(); ++c) luts[c].assign(lw.begin() + c * mod, lw.begin() + (c + 1) * mod);
                if (api == "vector") {
                    res = s.cc.EvalFunc(ct, luts);
                } else {
                    for (size_t c = 0; c < ct.size(); ++c) res.push_back(s.cc.EvalFunc(ct[c], luts[c]));
                }
            }
        } else if (op == "floor") {
            uint32_t rb = (uint32_t)arg_u64("roundbits", 0);
            if (api == "vector") {
                res = s.cc.EvalFloor(ct, rb);
            } else {
                for (auto& c : ct) res.push_back(s.cc.EvalFloor(c, rb));
            }
        } else if (op == "sign") {
            if (api == "vector") {
                res = s.cc.EvalSign(ct);
            } else {
                for (auto& c : ct) res.push_back(s.cc.EvalSign(c));
            }
        } else if (op == "decomp") {
            if (api == "vector") {
                dres = s.cc.EvalDecomp(ct);
            } else {
                for (auto& c : ct) dres.push_back(s.cc.EvalDecomp(c));
            }
        } else {
            BINGATE g = gate_of(op);
            auto ct2 = read_cts(arg("in2"), s.n, mod);
            if (api == "vector") {
                res = s.cc.EvalBinGate(g, ct, ct2);
            } else {
                for (size_t c = 0; c < ct.size(); ++c) res.push_back(s.cc.EvalBinGate(g, ct[c], ct2[c]));
            }
        }
        double dt = now_s() - ts;
        best = std::min(best, dt);
        total += dt;
        if (op == "decomp") {
            // both APIs return [ciphertext][digit] (vector: binfhe-base-scheme.cpp:1039-1085).
            // Written as [B][D][n+1].
            size_t D = dres.empty() ? 0 : dres[0].size();
            size_t B = ct.size();
            extra = D;
            std::vector<uint64_t> mods;
            for (size_t c = 0; c < B; ++c)
                for (size_t d = 0; d < D; ++d) {
                    const auto& x = dres[c][d];
                    append_ct(out, x);
                    if (c == 0) mods.push_back(x->GetModulus().ConvertToInt());
                }
            if (rep + 1 == reps && si + 1 == sizes.size()) {
                js << ",\"moduli\":[";
                for (size_t d = 0; d < mods.size(); ++d) js << (d ? "," : "") << mods[d];
                js << "]";
            }
        } else {
            for (auto& c : res) append_ct(out, c);
            if (!res.empty() && rep + 1 == reps && si + 1 == sizes.size())
                js << ",\"out_mod\":" << res[0]->GetModulus().ConvertToInt();
        }
    }
    if (g_limit) sweep << (si ? "," : "") << "{\"B\":" << g_limit << ",\"best_s\":" << best << ",\"mean_s\":" << total / reps
                       << ",\"threads\":" << (nthreads.empty() ? 0 : nthreads[si]) << "}";
    }
    if (sizes.size() > 1 || sizes[0]) js << ",\"sweep\":[" << sweep.str() << "]";
    if (api == "vector" && !g_batch) s.cc.GPUClean();
    write_u64(arg("out"), out);
    js << ",\"api\":\"" << api << "\",\"reps\":" << reps << ",\"best_s\":" << best << ",\"mean_s\":" << total / reps
       << ",\"words\":" << out.size() << ",\"fnv\":\"" << hex64(fnv1a64(out.data(), out.size())) << "\"";
    if (op == "decomp") js << ",\"digits\":" << extra;
    js << "}";
    printf("%s\n", js.str().c_str());
    return 0;
}
