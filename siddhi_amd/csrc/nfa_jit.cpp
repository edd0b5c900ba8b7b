// Query-specialised NFA kernels. The interpreter in kernels/nfa_impl.h serves every query from one build: it reads
// the plan (state table, filter and projection programs) from a device buffer, so every plan field is a dependent
// vector load, every plan loop and kind switch is a runtime branch, the filter programs run on an operand stack in
// scratch, and the lane's state is passed between non-inlined member functions through scratch frames.
//
// Here the same source is compiled (hiprtc, gfx950) once per query plan with the plan as a constant array
// (sm::kPlanBlob, SM_NFA_JIT): the plan's fields fold to constants, its loops unroll, kind switches drop their
// dead cases and the programs become straight-line code, so the whole interpreter inlines into one kernel. This
// is the device analogue of the reference compiling a query into its processor chain once, at app creation
// (SiddhiAppParser / QueryParser.parse, core/util/parser/QueryParser.java:79): the semantics are the
// interpreter's own, line for line; only the plan is fixed at compile time.
#include "nfa_jit.h"

#include <hip/hiprtc.h>
#include <dlfcn.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "nfa_jit_body.inc"  // kNfaJitBody (embed_jit.py)

#ifndef SM_ARCH
#define SM_ARCH "gfx950"  // the build's --offload-arch (Makefile ARCH)
#endif

namespace sm {

namespace {

struct JitKernel {
  hipModule_t mod = nullptr;
  hipFunction_t fn = nullptr;
};

std::mutex g_mu;
std::map<std::string, std::unique_ptr<JitKernel>>& cache() {
  static std::map<std::string, std::unique_ptr<JitKernel>> c;
  return c;
}

const char* kPrelude =
    "#define SM_NFA_JIT 1\n"
    // force the interpreter's member functions inline: with the plan constant they shrink to the plan's cases
    "#define SM_NFA_INLINE_PAR 1\n"
    "#define SM_NFA_INLINE_SMALL 1\n"
    "#define SM_NFA_INLINE_ADD 1\n"
    "#define SM_NFA_INLINE_FIRE 1\n"
    "#define SM_TIMER_INLINE 1\n"
    "typedef __hip_internal::int8_t int8_t;\n"
    "typedef __hip_internal::int16_t int16_t;\n"
    "typedef __hip_internal::int32_t int32_t;\n"
    "typedef __hip_internal::int64_t int64_t;\n"
    "typedef __hip_internal::uint8_t uint8_t;\n"
    "typedef __hip_internal::uint16_t uint16_t;\n"
    "typedef __hip_internal::uint32_t uint32_t;\n"
    "typedef __hip_internal::uint64_t uint64_t;\n"
    "#ifndef INT64_MAX\n#define INT64_MAX 9223372036854775807LL\n#endif\n"
    "#ifndef INT32_MAX\n#define INT32_MAX 2147483647\n#endif\n"
    "#ifndef INT32_MIN\n#define INT32_MIN (-2147483647 - 1)\n#endif\n"
    "#ifndef INT64_MIN\n#define INT64_MIN (-9223372036854775807LL - 1)\n#endif\n"
    "typedef struct ihipStream_t* hipStream_t;\n";

const char* kKernel = R"SMJIT(
extern "C" __global__ void __launch_bounds__(64) SM_NFA_JIT_ATTR sm_nfa_jit(sm::NfaBatch b, int64_t* ks_all, int64_t* heap_all,
                                                            int32_t heap_half, int64_t lanes, int32_t nkeys,
                                                            int32_t* err_out) {
  const int lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= nkeys) return;
  const int key = b.lane_perm ? (int)b.lane_perm[lane] : lane;
  sm::nfa_lane(b, nullptr, ks_all, heap_all, heap_half, lanes, key, err_out);
}
)SMJIT";

std::string blob_array(const std::vector<char>& blob) {
  std::ostringstream s;
  s << "namespace sm {\nstatic __device__ const unsigned char kPlanBlob[" << blob.size()
    << "] __attribute__((aligned(16))) = {";
  for (size_t i = 0; i < blob.size(); ++i) {
    if (i % 32 == 0) s << "\n";
    s << (unsigned)(unsigned char)blob[i] << ",";
  }
  s << "};\n}  // namespace sm\n";
  return s.str();
}

}  // namespace

std::string nfa_jit_source(const std::vector<char>& blob, bool lds, int compact) {
  std::string src = kPrelude;
  // Occupancy: room for 2 waves per SIMD (256 VGPRs). Measured on config 5 (N = 1e8, heap_words 1024, NFA kernel
  // ms): interpreter 74.3; JIT with the compiler's choice (268 VGPRs, 1 wave) 74.9, 2 waves 65.5, 4 waves 63.5;
  // with every event-path function inline, 4 waves 64.4, 3 waves 60.6. Round 3 (LDS-staged key state, no event
  // copies; config 5 plan): 3 waves = 168 VGPRs + 405 spilled (528 B of scratch per lane, 1e6 lanes: the spills
  // reach HBM, and under rocprofv3 the kernel ran 27 ms against 18 ms), 2 waves = 256 VGPRs + 32 spilled (144 B),
  // 1 wave = 288 with no scratch; NFA kernel 19.1 / 18.1 / 19.2 ms, 4 waves 20.4 ms. Default 2.
  // A/B: SM_NFA_JIT_WAVES=<n> (0 = no hint).
  const char* w = getenv("SM_NFA_JIT_WAVES");
  const int waves = w ? atoi(w) : 2;
  if (waves > 0)
    src += "#define SM_NFA_JIT_ATTR __attribute__((amdgpu_waves_per_eu(" + std::to_string(waves) + ")))\n";
  else
    src += "#define SM_NFA_JIT_ATTR\n";
  // every member function on the event path inline (A/B: SM_NFA_JIT_INLINE_ALL=0 leaves it to the compiler)
  const char* e = getenv("SM_NFA_JIT_INLINE_ALL");
  if (!e || atoi(e)) src += "#define SM_NFA_JIT_INLINE_ALL 1\n";
  if (lds) src += "#define SM_NFA_LDS 1\n";
  if (compact >= 0) src += "#define SM_LANE_COMPACT_CONST " + std::to_string(compact ? 1 : 0) + "\n";
  src += blob_array(blob);
  src += kNfaJitBody;
  src += kKernel;
  return src;
}

std::string nfa_jit_source(const std::vector<char>& blob, int compact) {
  return nfa_jit_source(blob, nfa_jit_lds_bytes(blob) > 0, compact);
}

bool nfa_jit_lds() {
  static const char* env = getenv("SM_NFA_JIT_LDS");
  return !env || atoi(env) != 0;
}

namespace {
// LDS a workgroup may allocate on the current device (0 without a device: the build check then assumes it fits)
int64_t device_lds_limit() {
  int dev = 0, v = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess) return 0;
  return v;
}
}  // namespace

int64_t nfa_jit_lds_bytes(const std::vector<char>& blob) {
  if (!nfa_jit_lds()) return 0;
  const DQuery* q = (const DQuery*)blob.data();
  const int64_t need = (int64_t)(q->ks_sched + 3) * 64 * 8;  // (pre words + post bits word + kNfaLdsMisc) x 64 lanes
  static const int64_t limit = device_lds_limit();
  // a plan whose staged key state exceeds the workgroup's LDS keeps it in HBM (the interpreter's layout)
  return limit > 0 && need > limit ? 0 : need;
}

bool nfa_jit_wanted(int option, int64_t records) {
  static const char* env = getenv("SM_NFA_JIT");
  if (env && *env) return atoi(env) != 0;
  if (option >= 0) return option != 0;
  return records >= (int64_t)1 << 20;  // the compile (seconds) pays off on large batches only
}

std::string nfa_jit_arch() {
  // the device's own target when one is visible (its gcnArchName without the feature suffix), else the build's
  int dev = 0;
  hipDeviceProp_t prop;
  if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess) {
    std::string a = prop.gcnArchName;
    a = a.substr(0, a.find(':'));
    if (a.rfind("gfx", 0) == 0) return a;
  }
  return SM_ARCH;
}

namespace {
// Code-object cache on disk: a plan's kernel takes minutes to compile (hiprtc, one thread), and every process that
// runs the plan (a test run, the bench, a profiler pass) would compile it again. The file name is a hash of
// everything the code depends on (HIP version, target, options, the whole source with the plan and the knobs), so
// a stale file is never picked up. Directory: SM_NFA_JIT_CACHE ("" = off), else jit_cache/ next to the library's
// lib/ directory (in-tree, so code objects compiled on the build host travel with the tree like the library;
// tools/jit_precompile.py fills it).
uint64_t fnv1a(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
  return h;
}
std::string jit_cache_dir() {
  if (const char* e = getenv("SM_NFA_JIT_CACHE")) return e;
  Dl_info info;
  if (!dladdr((void*)&fnv1a, &info) || !info.dli_fname) return "";
  std::string lib = info.dli_fname;
  const size_t slash = lib.rfind('/');
  if (slash == std::string::npos) return "";
  return lib.substr(0, slash) + "/../jit_cache";
}
}  // namespace

std::vector<char> nfa_jit_compile(const std::vector<char>& blob, int compact) {
  const std::string src = nfa_jit_source(blob, compact);
  if (const char* dump = getenv("SM_NFA_JIT_DUMP")) {
    if (FILE* f = fopen(dump, "w")) {
      fwrite(src.data(), 1, src.size(), f);
      fclose(f);
    }
  }
  const std::string arch = "--offload-arch=" + nfa_jit_arch();
  const char* opts[] = {arch.c_str(), "-O3", "-std=c++17", "-Wno-pass-failed"};
  const std::string dir = jit_cache_dir();
  std::string file;
  if (!dir.empty()) {
    // the hiprtc that is loaded, not the one built against: a process that imported torch first compiles with the
    // hiprtc and comgr torch bundles (ROCm 7.0 in this image), one without with /opt/rocm's (7.2), and the two make
    // different code from the same source (config-5 emitting variant: 170 VGPRs and 112 B of scratch, NFA kernel 108
    // ms, against 256 VGPRs and 192 B, 139 ms)
    int rtc_major = 0, rtc_minor = 0;
    hiprtcVersion(&rtc_major, &rtc_minor);
    char name[32];
    snprintf(name, sizeof name, "%016llx.co",
             (unsigned long long)fnv1a(std::to_string(HIP_VERSION) + "|" + std::to_string(rtc_major) + "." +
                                       std::to_string(rtc_minor) + "|" + opts[0] + "|" + opts[1] + "|" + opts[2] +
                                       "|" + opts[3] + "|" + src));
    file = dir + "/" + name;
    if (FILE* f = fopen(file.c_str(), "rb")) {
      std::vector<char> code;
      char buf[1 << 16];
      size_t r;
      while ((r = fread(buf, 1, sizeof buf, f)) > 0) code.insert(code.end(), buf, buf + r);
      fclose(f);
      if (!code.empty()) return code;
    }
  }
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "sm_nfa_jit.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS)
    throw std::runtime_error("nfa jit: hiprtcCreateProgram failed");
  const hiprtcResult rc = hiprtcCompileProgram(prog, 4, opts);
  if (rc != HIPRTC_SUCCESS) {
    size_t ls = 0;
    hiprtcGetProgramLogSize(prog, &ls);
    std::string log(ls + 1, '\0');
    hiprtcGetProgramLog(prog, &log[0]);
    hiprtcDestroyProgram(&prog);
    throw std::runtime_error("nfa jit: compile failed: " + log.substr(0, 4000));
  }
  size_t cs = 0;
  hiprtcGetCodeSize(prog, &cs);
  std::vector<char> code(cs);
  hiprtcGetCode(prog, code.data());
  hiprtcDestroyProgram(&prog);
  if (!file.empty()) {  // written under a private name, then renamed: readers never see a partial file
    mkdir(dir.c_str(), 0775);
    const std::string tmp = file + "." + std::to_string((long)getpid()) + ".tmp";
    if (FILE* f = fopen(tmp.c_str(), "wb")) {
      const bool ok = fwrite(code.data(), 1, code.size(), f) == code.size();
      if (fclose(f) == 0 && ok) rename(tmp.c_str(), file.c_str());
      else remove(tmp.c_str());
    }
  }
  return code;
}

void* nfa_jit_function(const std::vector<char>& blob, int compact) {
  int dev = 0;
  SM_HIP(hipGetDevice(&dev));
  const std::string key = std::to_string(dev) + ":" + nfa_jit_source(blob, compact);  // the source carries the knobs too
  {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = cache().find(key);
    if (it != cache().end()) return (void*)it->second->fn;
  }
  // compile (seconds) without holding the cache: other apps' queries keep launching their kernels meanwhile
  const std::vector<char> code = nfa_jit_compile(blob, compact);
  auto k = std::make_unique<JitKernel>();
  SM_HIP(hipModuleLoadData(&k->mod, code.data()));
  SM_HIP(hipModuleGetFunction(&k->fn, k->mod, "sm_nfa_jit"));
  std::lock_guard<std::mutex> g(g_mu);
  auto it = cache().find(key);
  if (it != cache().end()) {  // compiled concurrently by another thread: keep the first
    (void)hipModuleUnload(k->mod);
    return (void*)it->second->fn;
  }
  void* fn = (void*)k->fn;
  cache()[key] = std::move(k);
  return fn;
}

void launch_nfa_jit(void* fn, int64_t lds_bytes, const NfaBatch& b, int64_t* ks, int64_t* heap, int32_t heap_half,
                    int64_t lanes, int32_t nkeys, int32_t* err_dev, hipStream_t s) {
  if (nkeys <= 0) return;
  NfaBatch bb = b;
  void* args[] = {&bb, &ks, &heap, &heap_half, &lanes, &nkeys, &err_dev};
  const unsigned blocks = (unsigned)((nkeys + 63) / 64);
  SM_HIP(hipModuleLaunchKernel((hipFunction_t)fn, blocks, 1, 1, 64, 1, 1, (unsigned)lds_bytes, s, args, nullptr));
}

}  // namespace sm
