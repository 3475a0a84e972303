// jit.cpp — hipRTC specialisation of expression programs (see jit.h).
#include "jit.h"

#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "jit_src.h"  // build/jit_src.h: phys.h + vm.h + vm_device.h as one string

namespace mbx {
namespace jit {

namespace {

int Mode() {  // 0 off, 1 async, 2 sync
  const char *e = getenv("MBX_JIT");
  if (!e || !*e) return 1;
  if (!strcmp(e, "0") || !strcmp(e, "off")) return 0;
  if (!strcmp(e, "sync")) return 2;
  return 1;
}

// Shared kernel scaffolding: the same tile loop, selection bits and output
// stores as the interpreter kernels, around a generated straight-line body.
const char *kFilterHead = R"(
extern "C" __global__ __launch_bounds__(256) void mbx_jit_filter(mbx::VmProgram P, mbx::dev::VmCols C, int64_t nrows,
    int64_t rs, int64_t rstep, uint64_t *__restrict__ bits, uint32_t *__restrict__ tile_counts, int32_t *err) {
  using namespace mbx;
  using namespace mbx::dev;
  __shared__ uint32_t wcnt[4];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t ntiles = (nrows + VM_TILE - 1) / VM_TILE;
  VmCols Cs = C;
)";

const char *kProjectHead = R"(
extern "C" __global__ __launch_bounds__(256) void mbx_jit_project(mbx::VmProgram P, mbx::dev::VmCols C, int64_t nrows,
    int64_t rs, int64_t rstep, const uint64_t *__restrict__ bits, const int64_t *__restrict__ tile_off,
    mbx::dev::VmOuts O, int32_t *err) {
  using namespace mbx;
  using namespace mbx::dev;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t ntiles = (nrows + VM_TILE - 1) / VM_TILE;
  VmCols Cs = C;
)";

std::string Body(const VmProgram &p) {
  std::ostringstream o;
  for (int k = 0; k < p.n_ins; k++) {
    const VmIns &I = p.ins[k];
    o << "      vm_step(P, Cs, " << (int)I.op << ", " << (int)I.dst << ", " << (int)I.a << ", " << (int)I.b << ", "
      << (int)I.c << ", " << (int)I.aux << ", row, active, rs, rstep, R, err);\n";
  }
  return o.str();
}

struct Entry {
  enum State { PENDING, READY, FAILED } state = PENDING;
  hipModule_t mod = nullptr;
  hipFunction_t fn = nullptr;
  std::string log;
};

// Process-lifetime state (deliberately never destroyed: compile threads may
// still hold it during static destruction); pending compiles are joined at
// exit so no thread is inside hipRTC while the process tears down.
struct State {
  std::mutex mu;
  std::condition_variable cv;
  std::map<std::pair<int, std::string>, std::shared_ptr<Entry>> cache;  // (device, source) -> kernel
  std::vector<std::thread> threads;
};
State &S() {
  static State *s = new State();
  return *s;
}
void JoinAll() {
  std::vector<std::thread> ts;
  {
    std::lock_guard<std::mutex> lk(S().mu);
    ts.swap(S().threads);
  }
  for (auto &t : ts)
    if (t.joinable()) t.join();
}
#define g_mu (S().mu)
#define g_cv (S().cv)
#define g_cache (S().cache)

std::string CompileToCode(const std::string &src, std::vector<char> *code) {
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "mbx_jit.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS)
    return "hiprtcCreateProgram failed";
  const char *opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
  hiprtcResult r = hiprtcCompileProgram(prog, 3, opts);
  std::string log;
  size_t ls = 0;
  if (hiprtcGetProgramLogSize(prog, &ls) == HIPRTC_SUCCESS && ls > 1) {
    log.resize(ls);
    hiprtcGetProgramLog(prog, &log[0]);
  }
  if (r != HIPRTC_SUCCESS) {
    hiprtcDestroyProgram(&prog);
    return log.empty() ? std::string("hiprtcCompileProgram failed") : log;
  }
  if (code) {
    size_t n = 0;
    hiprtcGetCodeSize(prog, &n);
    code->resize(n);
    hiprtcGetCode(prog, code->data());
  }
  hiprtcDestroyProgram(&prog);
  return "";
}

void Build(int device, std::string src, bool filter, std::shared_ptr<Entry> e) {
  std::vector<char> code;
  std::string err = CompileToCode(src, &code);
  hipModule_t mod = nullptr;
  hipFunction_t fn = nullptr;
  if (err.empty()) {
    hipSetDevice(device);
    if (hipModuleLoadData(&mod, code.data()) != hipSuccess ||
        hipModuleGetFunction(&fn, mod, filter ? "mbx_jit_filter" : "mbx_jit_project") != hipSuccess) {
      (void)hipGetLastError();
      err = "hipModuleLoadData/GetFunction failed";
    }
  }
  std::lock_guard<std::mutex> lk(g_mu);
  e->mod = mod;
  e->fn = fn;
  e->log = err;
  e->state = err.empty() ? Entry::READY : Entry::FAILED;
  g_cv.notify_all();
}

// The compiled kernel for this source on the current device, or nullptr.
hipFunction_t Get(const std::string &src, bool filter) {
  const int mode = Mode();
  if (mode == 0) return nullptr;
  int device = 0;
  (void)hipGetDevice(&device);
  std::shared_ptr<Entry> e;
  bool start = false;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto key = std::make_pair(device, src);
    auto it = g_cache.find(key);
    if (it == g_cache.end()) {
      e = std::make_shared<Entry>();
      g_cache[key] = e;
      start = true;
    } else {
      e = it->second;
    }
  }
  if (start) {
    if (mode == 2) {
      Build(device, src, filter, e);
    } else {
      static bool registered = (atexit(JoinAll), true);
      (void)registered;
      std::lock_guard<std::mutex> lk(g_mu);
      S().threads.emplace_back(Build, device, src, filter, e);
      return nullptr;
    }
  }
  std::unique_lock<std::mutex> lk(g_mu);
  if (mode == 2) g_cv.wait(lk, [&] { return e->state != Entry::PENDING; });
  return e->state == Entry::READY ? e->fn : nullptr;
}

}  // namespace

std::string Source(const VmProgram &p, const dev::VmCols &cols, bool filter) {
  std::ostringstream o;
  o << kJitPrelude;
  o << "\nstruct LocalRF {\n  int64_t l[" << (p.n_regs > 0 ? p.n_regs : 1) << "], h["
    << (p.n_regs > 0 ? p.n_regs : 1) << "];\n  uint8_t n[" << (p.n_regs > 0 ? p.n_regs : 1)
    << "];\n  __device__ __forceinline__ int64_t &lo(int i) { return l[i]; }\n"
       "  __device__ __forceinline__ int64_t &hi(int i) { return h[i]; }\n"
       "  __device__ __forceinline__ uint8_t &nl(int i) { return n[i]; }\n};\n";
  o << (filter ? kFilterHead : kProjectHead);
  // column physical types are part of the specialisation
  for (int q = 0; q < cols.n; q++) o << "  Cs.c[" << q << "].phys = " << cols.c[q].phys << ";\n";
  if (filter) {
    o << "  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {\n"
         "    const int64_t row = tile * VM_TILE + t;\n"
         "    const bool active = row < nrows;\n"
         "    LocalRF R = {};\n    {\n";
    o << Body(p);
    o << "    }\n"
         "    const bool sel = active && !R.nl(" << (int)p.pred_reg << ") && R.lo(" << (int)p.pred_reg << ") != 0;\n"
         "    const uint64_t m = __ballot(sel);\n"
         "    if (lane == 0) {\n      bits[tile * 4 + w] = m;\n      wcnt[w] = (uint32_t)__popcll(m);\n    }\n"
         "    __syncthreads();\n"
         "    if (t == 0) tile_counts[tile] = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];\n"
         "    __syncthreads();\n  }\n}\n";
  } else {
    o << "  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {\n"
         "    const int64_t row = tile * VM_TILE + t;\n"
         "    bool sel;\n    int64_t out_idx;\n"
         "    if (bits) {\n"
         "      const uint64_t *tb = bits + tile * 4;\n"
         "      const uint64_t b0 = tb[0], b1 = tb[1], b2 = tb[2], b3 = tb[3];\n"
         "      if ((b0 | b1 | b2 | b3) == 0) continue;\n"
         "      const uint64_t mine = w == 0 ? b0 : w == 1 ? b1 : w == 2 ? b2 : b3;\n"
         "      const int before = (w > 0 ? __popcll(b0) : 0) + (w > 1 ? __popcll(b1) : 0) + (w > 2 ? __popcll(b2) : 0);\n"
         "      sel = (mine >> lane) & 1ull;\n"
         "      const uint64_t lt = lane ? (mine & ((1ull << lane) - 1ull)) : 0ull;\n"
         "      out_idx = tile_off[tile] + before + __popcll(lt);\n"
         "    } else {\n      sel = row < nrows;\n      out_idx = row;\n    }\n"
         "    const bool active = sel;\n"
         "    LocalRF R = {};\n    {\n";
    o << Body(p);
    o << "    }\n    if (sel) {\n";
    for (int q = 0; q < p.n_out; q++) {
      const int r = p.out_reg[q];
      o << "      store_phys(O.data[" << q << "], " << (int)p.out_phys[q] << ", out_idx, R.lo(" << r << "), R.hi(" << r
        << "));\n"
           "      if (R.nl(" << r << ") && O.nullbits[" << q << "]) {\n"
           "        atomicOr(&O.nullbits[" << q << "][out_idx >> 5], 1u << (out_idx & 31));\n"
           "        if (O.anynull) O.anynull[" << q << "] = 1;\n      }\n";
    }
    o << "    }\n  }\n}\n";
  }
  return o.str();
}

std::string CompileCheck(const std::string &src) { return CompileToCode(src, nullptr); }

static int GridFor(int64_t ntiles) {
  int cus = 0, d = 0;
  (void)hipGetDevice(&d);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, d);
  if (cus <= 0) cus = 256;
  int64_t g = ntiles < 1 ? 1 : ntiles;
  if (g > (int64_t)cus * 8) g = (int64_t)cus * 8;
  return (int)g;
}

bool VmFilter(const VmProgram &p, const dev::VmCols &cols, int64_t nrows, int64_t range_start, int64_t range_step,
              uint64_t *sel_bits, uint32_t *tile_counts, int32_t *err, hipStream_t s) {
  if (nrows <= 0) return false;
  hipFunction_t fn = Get(Source(p, cols, true), true);
  if (!fn) return false;
  VmProgram P = p;
  dev::VmCols C = cols;
  void *args[] = {&P, &C, &nrows, &range_start, &range_step, &sel_bits, &tile_counts, &err};
  const int64_t ntiles = (nrows + VM_TILE - 1) / VM_TILE;
  return hipModuleLaunchKernel(fn, GridFor(ntiles), 1, 1, 256, 1, 1, 0, s, args, nullptr) == hipSuccess;
}

bool VmProject(const VmProgram &p, const dev::VmCols &cols, int64_t nrows, int64_t range_start, int64_t range_step,
               const uint64_t *sel_bits, const int64_t *tile_offsets, const dev::VmOuts &outs, int32_t *err,
               hipStream_t s) {
  if (nrows <= 0) return false;
  hipFunction_t fn = Get(Source(p, cols, false), false);
  if (!fn) return false;
  VmProgram P = p;
  dev::VmCols C = cols;
  dev::VmOuts O = outs;
  void *args[] = {&P, &C, &nrows, &range_start, &range_step, &sel_bits, &tile_offsets, &O, &err};
  const int64_t ntiles = (nrows + VM_TILE - 1) / VM_TILE;
  return hipModuleLaunchKernel(fn, GridFor(ntiles), 1, 1, 256, 1, 1, 0, s, args, nullptr) == hipSuccess;
}

}  // namespace jit
}  // namespace mbx
