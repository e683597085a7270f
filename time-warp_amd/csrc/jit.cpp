// jit.cpp — the scenario compiler of libtimewarp.so (tw_set_jit).
//
// A scenario's thread programs (the lowered handler state machines of
// timewarp/program.py, include/timewarp.h's ISA) are fixed at tw_load.  The
// interpreter of engine_dev.hpp decodes every instruction on every pass:
// per-lane image fetch from LDS, operand and uop-class decode, select chains
// over the register-result classes, an LDS register file.  Here the image is
// turned into device code instead: one call of Lane::jop<word, imm> per pc,
// in program order, inside a switch on the first running lane's pc
// (tw_jit_dispatch), so every operand, uop class and register index is a
// compile-time constant and a straight-line run of instructions falls through
// from one case into the next while some lane continues there.  The running
// thread's registers stay in VGPRs (Lane::rg/rs).
//
// The generated source is appended to the engine's own device source
// (engine_dev.hpp, embedded into the library by embed_src.py) and compiled
// with hiprtc for gfx950 -- in process, no compiler binary is run.  Results
// are bit-identical to the interpreter's: both run Lane::pass, with the same
// semantics per instruction (TimedT.hs:234-376 as restated in DESIGN.md §1).
//
// The reference compiles its scenarios too: they are Haskell code built by
// GHC; this is the same step for the lowered form.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "../../include/timewarp.h"
#include "jit.hpp"
#include "jit_src.inc"

namespace tw {

namespace {

// the hiprtc compile brings no C library headers: the fixed-width types come
// from hiprtc's own runtime header (namespace __hip_internal)
const char* kPrelude =
    "#include <hip/hip_runtime.h>\n"
    "using __hip_internal::uint8_t; using __hip_internal::uint16_t; using __hip_internal::uint32_t;\n"
    "using __hip_internal::uint64_t; using __hip_internal::int8_t; using __hip_internal::int16_t;\n"
    "using __hip_internal::int32_t; using __hip_internal::int64_t; using __hip_internal::size_t;\n"
    "#define INT64_MAX 0x7fffffffffffffffLL\n"
    "#define INT64_MIN (-INT64_MAX - 1LL)\n"
    "#define UINT64_MAX 0xffffffffffffffffULL\n";

uint64_t fnv1a(const std::string& s, uint64_t h = 1469598103934665603ull) {
    for (unsigned char ch : s) h = (h ^ ch) * 1099511628211ull;
    return h;
}

std::string imm_lit(int32_t v) {
    if (v == INT32_MIN) return "(-2147483647 - 1)";
    return std::to_string(v);
}

// The per-scenario part: the block dispatch over every pc of the image.  Each
// instruction is its own specialised code (Lane::jop: the front end emits only
// its uop class, or its one case of the rare-op switch), falling through to
// the next pc while some lane continues there.  The heavy rare ops (throwTo,
// throw, the timeout watchdog: each would inline the queue re-stamp or the
// unwinder again) jump to one shared interpreter pass after the switch
// (Lane::jrare).
bool shared_op(uint32_t w0) {
    const uint32_t op = w0 & 0xFFu;
    const char* env = getenv("TW_JIT_SHARED");  // (experiments: a comma list of opcodes)
    if (env && *env) {
        std::string e = std::string(",") + env + ",";
        return e.find("," + std::to_string(op) + ",") != std::string::npos;
    }
    return op == TW_OP_THROW_TO || op == TW_OP_THROW || op == TW_OP_TMO_FIRE;
}

std::string dispatch_src(const tw_insn* insns, uint32_t n) {
    std::string s;
    s.reserve(128 * (size_t)n + 512);
    s += "#ifndef TW_JIT_DISPATCH_ATTR\n#define TW_JIT_DISPATCH_ATTR __forceinline__\n#endif\n";
    s += "namespace {\n"
         "template <class LT, class ST>\n"
         "__device__ TW_JIT_DISPATCH_ATTR void tw_jit_dispatch(LT& L, Th& th, uint32_t slot, ST& s, uint32_t fpc) {\n"
         "    switch (fpc) {\n";
    char buf[200];
    for (uint32_t pc = 0; pc < n; ++pc) {
        snprintf(buf, sizeof buf, "    case %uu: ", pc);
        s += buf;
        if (shared_op(insns[pc].w0)) {
            s += "goto rare;\n";
            continue;
        }
        snprintf(buf, sizeof buf, "L.template jop<0x%08xu, %s>(th, slot, s, %uu)", insns[pc].w0,
                 imm_lit(insns[pc].imm).c_str(), pc);
        if (pc + 1 < n) {
            s += "if (!";
            s += buf;
            if (shared_op(insns[pc + 1].w0)) {
                snprintf(buf, sizeof buf, ") break;\n        fpc = %uu;\n        goto rare;\n", pc + 1);
                s += buf;
            } else {
                s += ") break;\n        [[fallthrough]];\n";
            }
        } else {
            s += buf;
            s += ";\n        break;\n";
        }
    }
    s += "    default: L.jbad(s, fpc); break;\n"
         "    }\n"
         "    return;\n"
         "rare:\n"
         "    L.jrare(th, slot, s, fpc);\n"
         "}\n";
    return s;
}

struct Entry {
    std::string code;
    std::vector<std::string> names;
};
std::mutex g_mu;
std::map<uint64_t, Entry> g_cache;  // in-process: (source, options) -> code object

bool read_file(const std::string& p, std::string* out) {
    FILE* f = fopen(p.c_str(), "rb");
    if (!f) return false;
    std::string d;
    char b[65536];
    size_t k;
    while ((k = fread(b, 1, sizeof b, f)) > 0) d.append(b, k);
    fclose(f);
    *out = std::move(d);
    return true;
}
bool write_file(const std::string& p, const std::string& d) {
    const std::string tmp = p + ".tmp";
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f) return false;
    const bool ok = fwrite(d.data(), 1, d.size(), f) == d.size();
    fclose(f);
    return ok && rename(tmp.c_str(), p.c_str()) == 0;
}

}  // namespace

int jit_compile(const tw_insn* insns, uint32_t n_insns, const std::vector<std::string>& inst,
                const std::vector<std::string>& defs, std::string* code, std::vector<std::string>* names,
                double* compile_ms) {
    if (!insns || !n_insns || inst.empty() || !code || !names) return TW_ERR_INVALID;
    std::string src = kPrelude;
    src += kTwEngineSrc;
    src += "\n// ---- generated by jit.cpp: the scenario's instruction blocks\n";
    src += dispatch_src(insns, n_insns);
    std::vector<std::string> exprs;
    for (const std::string& a : inst) {
        const std::string e = "tw_run_kernel<" + a + ", true>";
        exprs.push_back(e);
        src += "template __global__ void " + e + "(Dev, int64_t, uint64_t, uint32_t);\n";
    }
    src += "}  // namespace\n";
    const char* rocm = getenv("ROCM_PATH");
    std::vector<std::string> opts = {"--offload-arch=gfx950", "-O3", "-std=c++17",
                                     std::string("-I") + (rocm && *rocm ? rocm : "/opt/rocm") + "/include"};
    for (const std::string& d : defs) opts.push_back(d);
    if (const char* x = getenv("TW_JIT_OPTS")) {  // (experiments: extra options, space-separated)
        std::string o;
        for (const char* p = x;; ++p) {
            if (*p == ' ' || *p == 0) {
                if (!o.empty()) opts.push_back(o);
                o.clear();
                if (!*p) break;
            } else {
                o += *p;
            }
        }
    }
    std::string key_s = src;
    for (const std::string& o : opts) key_s += "\n" + o;
    const uint64_t key = fnv1a(key_s);
    *compile_ms = 0.0;
    {
        std::lock_guard<std::mutex> g(g_mu);
        auto it = g_cache.find(key);
        if (it != g_cache.end()) {
            *code = it->second.code;
            *names = it->second.names;
            return TW_OK;
        }
    }
    // optional on-disk cache (TW_JIT_CACHE=dir): code object + lowered names
    const char* cdir = getenv("TW_JIT_CACHE");
    char hex[32];
    snprintf(hex, sizeof hex, "%016llx", (unsigned long long)key);
    if (cdir && *cdir) {
        std::string co, nm;
        if (read_file(std::string(cdir) + "/" + hex + ".co", &co) && read_file(std::string(cdir) + "/" + hex + ".names", &nm)) {
            std::vector<std::string> ns;
            size_t p = 0;
            while (p < nm.size()) {
                size_t q = nm.find('\n', p);
                if (q == std::string::npos) q = nm.size();
                if (q > p) ns.push_back(nm.substr(p, q - p));
                p = q + 1;
            }
            if (ns.size() == exprs.size() && !co.empty()) {
                std::lock_guard<std::mutex> g(g_mu);
                g_cache[key] = Entry{co, ns};
                *code = co;
                *names = ns;
                return TW_OK;
            }
        }
    }
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "tw_scenario.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS)
        return TW_ERR_JIT;
    for (const std::string& e : exprs) hiprtcAddNameExpression(prog, e.c_str());
    std::vector<const char*> ov;
    for (const std::string& o : opts) ov.push_back(o.c_str());
    const auto t0 = std::chrono::steady_clock::now();
    const hiprtcResult r = hiprtcCompileProgram(prog, (int)ov.size(), ov.data());
    *compile_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (r != HIPRTC_SUCCESS) {
        size_t ls = 0;
        hiprtcGetProgramLogSize(prog, &ls);
        std::string log(ls + 1, '\0');
        hiprtcGetProgramLog(prog, &log[0]);
        fprintf(stderr, "timewarp: scenario compile failed (%s):\n%.4000s\n", hiprtcGetErrorString(r), log.c_str());
        hiprtcDestroyProgram(&prog);
        return TW_ERR_JIT;
    }
    std::vector<std::string> ns;
    for (const std::string& e : exprs) {
        const char* low = nullptr;
        if (hiprtcGetLoweredName(prog, e.c_str(), &low) != HIPRTC_SUCCESS || !low) {
            hiprtcDestroyProgram(&prog);
            return TW_ERR_JIT;
        }
        ns.push_back(low);
    }
    size_t cs = 0;
    if (hiprtcGetCodeSize(prog, &cs) != HIPRTC_SUCCESS || cs == 0) {
        hiprtcDestroyProgram(&prog);
        return TW_ERR_JIT;
    }
    std::string co(cs, '\0');
    hiprtcGetCode(prog, &co[0]);
    hiprtcDestroyProgram(&prog);
    if (const char* dump = getenv("TW_JIT_DUMP")) {  // (inspection: the source and the code object)
        (void)write_file(std::string(dump) + ".hip", src);
        (void)write_file(std::string(dump) + ".co", co);
    }
    if (cdir && *cdir) {
        std::string nm;
        for (const std::string& x : ns) nm += x + "\n";
        (void)write_file(std::string(cdir) + "/" + hex + ".co", co);
        (void)write_file(std::string(cdir) + "/" + hex + ".names", nm);
    }
    {
        std::lock_guard<std::mutex> g(g_mu);
        g_cache[key] = Entry{co, ns};
    }
    *code = std::move(co);
    *names = std::move(ns);
    return TW_OK;
}

}  // namespace tw
