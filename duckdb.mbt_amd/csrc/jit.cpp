// jit.cpp — hipRTC specialisation of expression programs (see jit.h).
#include "jit.h"

#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <condition_variable>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "jit_src.h"  // build/jit_src.h: phys.h + vm.h + vm_device.h as one string
#include "types.h"
#include "knobs.h"

namespace mbx {
namespace jit {

namespace {

int Mode() {  // 0 off, 1 async, 2 sync
  const char *e = Knob("MBX_JIT");
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

// Column loads of a program for one row, hoisted ahead of all arithmetic
// (the loads of every row a thread handles are then in flight together; the
// values wait in L<k>l/h/n<sfx> until the V_LOADCOL that consumes them).
std::string Preload(const VmProgram &p, const std::string &sfx, const std::string &lrow, const std::string &act) {
  std::ostringstream o;
  for (int k = 0; k < p.n_ins; k++) {
    const VmIns &I = p.ins[k];
    if (I.op != V_LOADCOL) continue;
    o << "    int64_t L" << k << "l" << sfx << ", L" << k << "h" << sfx << ";\n"
      << "    load_phys(Cs.c[" << (int)I.a << "].data, Cs.c[" << (int)I.a << "].phys, " << lrow << ", L" << k << "l"
      << sfx << ", L" << k << "h" << sfx << ");\n"
      << "    const uint8_t L" << k << "n" << sfx << " = (" << act << " && bit_valid(Cs.c[" << (int)I.a << "].validity, "
      << lrow << ")) ? 0 : 1;\n";
  }
  return o.str();
}

std::string Body(const VmProgram &p, const std::string &sfx = "") {
  std::ostringstream o;
  for (int k = 0; k < p.n_ins; k++) {
    const VmIns &I = p.ins[k];
    if (I.op == V_LOADCOL) {
      o << "      R.lo(" << (int)I.dst << ") = L" << k << "l" << sfx << "; R.hi(" << (int)I.dst << ") = L" << k << "h" << sfx
        << "; R.nl(" << (int)I.dst << ") = L" << k << "n" << sfx << ";\n";
      continue;
    }
    o << "      vm_step<LocalRF, true>(P, Cs, " << (int)I.op << ", " << (int)I.dst << ", " << (int)I.a << ", "
      << (int)I.b << ", " << (int)I.c << ", " << (int)I.aux << ", lrow, active, rs, rstep, R, err);\n";
  }
  return o.str();
}

// column physical types and the absence of NULL bitmaps are compiled in
void Specialise(std::ostringstream &o, const dev::VmCols &cols) {
  for (int q = 0; q < cols.n; q++) {
    o << "  Cs.c[" << q << "].phys = " << cols.c[q].phys << ";\n";
    if (!cols.c[q].validity) o << "  Cs.c[" << q << "].validity = nullptr;\n";
  }
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

void Build(int device, std::string src, std::string name, std::shared_ptr<Entry> e) {
  std::vector<char> code;
  std::string err = CompileToCode(src, &code);
  hipModule_t mod = nullptr;
  hipFunction_t fn = nullptr;
  if (err.empty()) {
    hipSetDevice(device);
    if (hipModuleLoadData(&mod, code.data()) != hipSuccess ||
        hipModuleGetFunction(&fn, mod, name.c_str()) != hipSuccess) {
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

// The compiled kernel `name` of this source on the current device, or nullptr.
hipFunction_t GetNamed(const std::string &src, const std::string &name) {
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
      Build(device, src, name, e);
    } else {
      static bool registered = (atexit(JoinAll), true);
      (void)registered;
      std::lock_guard<std::mutex> lk(g_mu);
      S().threads.emplace_back(Build, device, src, name, e);
      return nullptr;
    }
  }
  std::unique_lock<std::mutex> lk(g_mu);
  if (mode == 2) g_cv.wait(lk, [&] { return e->state != Entry::PENDING; });
  return e->state == Entry::READY ? e->fn : nullptr;
}

hipFunction_t Get(const std::string &src, bool filter) {
  return GetNamed(src, filter ? "mbx_jit_filter" : "mbx_jit_project");
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
  Specialise(o, cols);
  if (filter) {
    o << "  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {\n"
         "    const int64_t row = tile * VM_TILE + t;\n"
         "    const bool active = row < nrows;\n"
         "    const int64_t lrow = active ? row : nrows - 1;\n";
    o << Preload(p, "", "lrow", "active");
    o << "    LocalRF R = {};\n    {\n";
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
         "    const int64_t lrow = row < nrows ? row : nrows - 1;\n";
    o << Preload(p, "", "lrow", "active");
    o << "    LocalRF R = {};\n    {\n";
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

bool Enabled() { return Mode() != 0; }

// Source of the fused aggregate kernel (see jit.h, VmAggregate).
static std::string AggSource(const VmProgram &p, const dev::VmCols &cols) {
  std::ostringstream o;
  const int nr = p.n_regs > 0 ? p.n_regs : 1;
  o << kJitPrelude;
  o << "\nstruct LocalRF {\n  int64_t l[" << nr << "], h[" << nr << "];\n  uint8_t n[" << nr
    << "];\n  __device__ __forceinline__ int64_t &lo(int i) { return l[i]; }\n"
       "  __device__ __forceinline__ int64_t &hi(int i) { return h[i]; }\n"
       "  __device__ __forceinline__ uint8_t &nl(int i) { return n[i]; }\n};\n"
       "struct JAggState {\n  unsigned long long count, sum_lo;\n  long long sum_hi, min_i, max_i;\n  double sum_f;\n"
       "  unsigned long long min_f, max_f;\n};\n"
       "__device__ __forceinline__ unsigned long long jshfl(unsigned long long v, int m) {\n"
       "  return (unsigned long long)__shfl_xor((long long)v, m, 64);\n}\n";
  o << "extern \"C\" __global__ __launch_bounds__(256) void mbx_jit_agg(mbx::VmProgram P, mbx::dev::VmCols C, "
       "int64_t nrows, int64_t rs, int64_t rstep, JAggState *states, unsigned long long *cstar, int32_t *err) {\n"
       "  using namespace mbx;\n  using namespace mbx::dev;\n  VmCols Cs = C;\n";
  Specialise(o, cols);
  o << "  unsigned long long cs = 0;\n";
  for (int j = 0; j < p.n_out; j++) {
    if (p.out_reg[j] == 255) continue;
    if (p.out_class[j] == VC_F64)
      o << "  unsigned long long c" << j << " = 0, fmn" << j << " = ~0ull, fmx" << j << " = 0;\n  double sf" << j
        << " = 0;\n";
    else
      o << "  unsigned long long c" << j << " = 0, slo" << j << " = 0;\n  long long shi" << j << " = 0, mn" << j
        << " = INT64_MAX, mx" << j << " = INT64_MIN;\n";
  }
  // Rows per thread and iteration: NR independent register files, so the
  // column loads of all NR rows are in flight together.  Default: U single
  // rows strided by the grid.  MBX_JIT_PAIRS=1: U pairs of consecutive rows,
  // an 8-byte (4-byte) column of a full pair fetched with ONE 16-byte (8-byte)
  // load -- measured no faster (profiles/r01_jit_sweep.log), kept for sweeps.
  int U = 4;
  if (const char *e = Knob("MBX_JIT_U")) U = atoi(e) == 1 || atoi(e) == 2 || atoi(e) == 8 ? atoi(e) : 4;
  const char *pe = Knob("MBX_JIT_PAIRS");
  const bool pairs = pe && strcmp(pe, "1") == 0;
  const int NR = pairs ? 2 * U : U;
  const int64_t span = pairs ? 2 : 1;
  o << "  const int64_t S = (int64_t)gridDim.x * blockDim.x;\n"
       "  const int64_t nunits = (nrows + " << span - 1 << ") / " << span << ";\n"
       "  for (int64_t base = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; base < nunits; base += " << U << " * S) {\n";
  for (int u = 0; u < U; u++) {
    o << "    const int64_t unit" << u << " = base + " << u << " * S;\n";
    for (int h = 0; h < span; h++) {
      const int r = u * span + h;
      o << "    const int64_t row" << r << " = unit" << u << " * " << span << " + " << h << ";\n    const bool act" << r
        << " = row" << r << " < nrows;\n    const int64_t lrow" << r << " = act" << r << " ? row" << r
        << " : nrows - 1;\n    LocalRF R" << r << " = {};\n";
    }
  }
  if (pairs) {
    for (int u = 0; u < U; u++) {
      const std::string a = std::to_string(2 * u), b = std::to_string(2 * u + 1);
      o << "    const bool full" << u << " = act" << b << ";\n";
      for (int k = 0; k < p.n_ins; k++) {
        const VmIns &I = p.ins[k];
        if (I.op != V_LOADCOL) continue;
        const int ph = cols.c[I.a].phys;
        const bool nov = cols.c[I.a].validity == nullptr;
        const std::string ca = "Cs.c[" + std::to_string((int)I.a) + "]";
        o << "    int64_t L" << k << "l" << a << ", L" << k << "h" << a << ", L" << k << "l" << b << ", L" << k << "h" << b
          << ";\n";
        const char *vt = (ph == P_I64 || ph == P_F64 || ph == P_U64) ? "long long" : ph == P_I32 ? "int" : nullptr;
        if (vt && nov) {
          o << "    if (full" << u << ") {\n      typedef " << vt << " vv __attribute__((ext_vector_type(2)));\n"
            << "      const vv t = ((const vv *)" << ca << ".data)[unit" << u << "];\n"
            << "      L" << k << "l" << a << " = (long long)t.x; L" << k << "l" << b << " = (long long)t.y;\n";
          if (ph == P_U64)
            o << "      L" << k << "h" << a << " = 0; L" << k << "h" << b << " = 0;\n";
          else if (ph == P_F64)
            o << "      L" << k << "h" << a << " = 0; L" << k << "h" << b << " = 0;\n";
          else
            o << "      L" << k << "h" << a << " = L" << k << "l" << a << " >> 63; L" << k << "h" << b << " = L" << k << "l"
              << b << " >> 63;\n";
          o << "    } else {\n";
        } else {
          o << "    {\n";
        }
        o << "      load_phys(" << ca << ".data, " << ca << ".phys, lrow" << a << ", L" << k << "l" << a << ", L" << k << "h"
          << a << ");\n      load_phys(" << ca << ".data, " << ca << ".phys, lrow" << b << ", L" << k << "l" << b << ", L"
          << k << "h" << b << ");\n    }\n";
        o << "    const uint8_t L" << k << "n" << a << " = (act" << a << " && bit_valid(" << ca << ".validity, lrow" << a
          << ")) ? 0 : 1;\n    const uint8_t L" << k << "n" << b << " = (act" << b << " && bit_valid(" << ca
          << ".validity, lrow" << b << ")) ? 0 : 1;\n";
      }
    }
  } else {
    for (int r = 0; r < NR; r++)
      o << Preload(p, std::to_string(r), "lrow" + std::to_string(r), "act" + std::to_string(r));
  }
  for (int r = 0; r < NR; r++) {
    o << "    {\n      const int64_t lrow = lrow" << r << ";\n      const bool active = act" << r
      << ";\n      LocalRF &R = R" << r << ";\n";
    o << Body(p, std::to_string(r));
    o << "    }\n";
  }
  o << "#pragma unroll\n    for (int u = 0; u < " << NR << "; u++) {\n      LocalRF &R = ";
  for (int r = 0; r < NR - 1; r++) o << "u == " << r << " ? R" << r << " : ";
  o << "R" << NR - 1 << ";\n      const bool act = ";
  for (int r = 0; r < NR - 1; r++) o << "u == " << r << " ? act" << r << " : ";
  o << "act" << NR - 1 << ";\n";
  if (p.pred_reg != 255)
    o << "    const bool sel = act && !R.nl(" << (int)p.pred_reg << ") && R.lo(" << (int)p.pred_reg << ") != 0;\n";
  else
    o << "    const bool sel = act;\n";
  o << "    cs += sel;\n";
  for (int j = 0; j < p.n_out; j++) {
    const int r = p.out_reg[j];
    if (r == 255) continue;
    // bit0: sum, bit1: min/max.  All statistics by default: the lean variant
    // (only what the aggregate kind needs) measured 1.6x slower at 1e8 rows,
    // the scheduler sinks the hoisted loads when the loop body is short
    // (profiles/r01_jit_sweep.log); MBX_JIT_LEAN=1 selects it.
    int need = 3;
    if (Knob("MBX_JIT_LEAN") && p.out_phys[j]) need = p.out_phys[j];
    o << "    if (sel && !R.nl(" << r << ")) {\n      c" << j << "++;\n";
    if (p.out_class[j] == VC_F64) {
      o << "      const double d = __longlong_as_double(R.lo(" << r << "));\n";
      if (need & 1) o << "      sf" << j << " += d;\n";
      if (need & 2)
        o << "      const unsigned long long k = f64_order(d);\n      fmn" << j << " = k < fmn" << j << " ? k : fmn" << j
          << ";\n      fmx" << j << " = k > fmx" << j << " ? k : fmx" << j << ";\n";
    } else {
      o << "      const long long v = R.lo(" << r << "), vh = R.hi(" << r << ");\n";
      if (need & 1)
        o << "      const unsigned long long nlo = slo" << j << " + (unsigned long long)v;\n"
             "      shi" << j << " += vh + (nlo < slo" << j << " ? 1 : 0);\n      slo" << j << " = nlo;\n";
      if (need & 2)
        o << "      mn" << j << " = v < mn" << j << " ? v : mn" << j << ";\n      mx" << j << " = v > mx" << j << " ? v : mx" << j
          << ";\n";
    }
    o << "    }\n";
  }
  o << "    }\n  }\n";
  // Reduce every running statistic over the wave (shuffles), then over the
  // block's four waves (LDS), so each block issues ONE set of atomics: with
  // 2048 blocks the per-wave variant spent a visible part of the kernel on
  // same-address atomics.  Kinds: 0 u64 add, 1 s64 min, 2 s64 max, 3 f64 add,
  // 4 u64 min, 5 u64 max, 6 int128 add (lo, hi in two slots).
  struct RV { std::string lo, hi; int kind; };
  std::vector<RV> rv = {{"cs", "", 0}};
  for (int j = 0; j < p.n_out; j++) {
    if (p.out_reg[j] == 255) continue;
    const std::string J = std::to_string(j);
    rv.push_back({"c" + J, "", 0});
    if (p.out_class[j] == VC_F64) {
      rv.push_back({"sf" + J, "", 3});
      rv.push_back({"fmn" + J, "", 4});
      rv.push_back({"fmx" + J, "", 5});
    } else {
      rv.push_back({"slo" + J, "shi" + J, 6});
      rv.push_back({"mn" + J, "", 1});
      rv.push_back({"mx" + J, "", 2});
    }
  }
  // combine (x, xh) <- (x, xh) op (y, yh); y/yh are expressions of 64-bit bits
  auto comb = [&](const RV &v, const std::string &y, const std::string &yh) {
    const std::string &x = v.lo;
    switch (v.kind) {
      case 0: return "    " + x + " += " + y + ";\n";
      case 1: return "    { const long long t = (long long)(" + y + "); " + x + " = t < " + x + " ? t : " + x + "; }\n";
      case 2: return "    { const long long t = (long long)(" + y + "); " + x + " = t > " + x + " ? t : " + x + "; }\n";
      case 3: return "    " + x + " += __longlong_as_double((long long)(" + y + "));\n";
      case 4: return "    { const unsigned long long t = " + y + "; " + x + " = t < " + x + " ? t : " + x + "; }\n";
      case 5: return "    { const unsigned long long t = " + y + "; " + x + " = t > " + x + " ? t : " + x + "; }\n";
      default:
        return "    { const unsigned long long t = " + y + "; const long long th = (long long)(" + yh +
               "); const unsigned long long s2 = " + x + " + t; " + v.hi + " += th + (s2 < " + x + " ? 1 : 0); " + x +
               " = s2; }\n";
    }
  };
  auto bits = [](const RV &v, const std::string &x) {
    return v.kind == 3 ? "(unsigned long long)__double_as_longlong(" + x + ")" : "(unsigned long long)" + x;
  };
  int nslot = 0;
  for (const RV &v : rv) nslot += v.kind == 6 ? 2 : 1;
  o << "  for (int m = 32; m >= 1; m >>= 1) {\n";
  for (const RV &v : rv)
    o << comb(v, "jshfl(" + bits(v, v.lo) + ", m)", v.kind == 6 ? "jshfl(" + bits(v, v.hi) + ", m)" : "");
  o << "  }\n  __shared__ unsigned long long jred[4][" << nslot << "];\n  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;\n"
    << "  if (lane == 0) {\n";
  {
    int k = 0;
    for (const RV &v : rv) {
      o << "    jred[wv][" << k++ << "] = " << bits(v, v.lo) << ";\n";
      if (v.kind == 6) o << "    jred[wv][" << k++ << "] = " << bits(v, v.hi) << ";\n";
    }
  }
  o << "  }\n  __syncthreads();\n  if (threadIdx.x != 0) return;\n  for (int w = 1; w < (int)(blockDim.x >> 6); w++) {\n";
  {
    int k = 0;
    for (const RV &v : rv) {
      const std::string y = "jred[w][" + std::to_string(k++) + "]";
      const std::string yh = v.kind == 6 ? "jred[w][" + std::to_string(k++) + "]" : "";
      o << comb(v, y, yh);
    }
  }
  o << "  }\n";
  o << "  {\n    if (cs) atomicAdd(cstar, cs);\n";
  for (int j = 0; j < p.n_out; j++) {
    if (p.out_reg[j] == 255) continue;
    o << "    if (c" << j << ") {\n      JAggState *st = states + " << j << ";\n      atomicAdd(&st->count, c" << j << ");\n";
    if (p.out_class[j] == VC_F64) {
      o << "      atomicAdd(&st->sum_f, sf" << j << ");\n      atomicMin(&st->min_f, fmn" << j
        << ");\n      atomicMax(&st->max_f, fmx" << j << ");\n";
    } else {
      o << "      const unsigned long long old = atomicAdd(&st->sum_lo, slo" << j << ");\n"
           "      const unsigned long long carry = (old + slo" << j << ") < old ? 1ull : 0ull;\n"
           "      atomicAdd((unsigned long long *)&st->sum_hi, (unsigned long long)shi" << j << " + carry);\n"
           "      atomicMin(&st->min_i, mn" << j << ");\n      atomicMax(&st->max_i, mx" << j << ");\n";
    }
    o << "    }\n";
  }
  o << "  }\n}\n";
  return o.str();
}

std::string AggSourceForTest(const VmProgram &p, const dev::VmCols &cols) { return AggSource(p, cols); }

// ---- fused GROUP BY (jit.h, VmGroupAggregate) ------------------------------

// Kernel argument mirror of the generated `struct JGroup`.
struct JGroupArg {
  int64_t kmin[JIT_MAX_KEYS], radix[JIT_MAX_KEYS], stride[JIT_MAX_KEYS];
  int32_t nslots, R;
};

static bool ArgSum(const VmProgram &p, int j) { return (p.out_phys[j] & 1) != 0; }
static bool ArgMM(const VmProgram &p, int j) { return (p.out_phys[j] & 2) != 0; }

size_t GroupLdsBytes(const VmProgram &p, int64_t nslots, int R) {
  const size_t ns = (size_t)nslots * R, a4 = (ns * 4 + 7) & ~(size_t)7;
  size_t b = a4;  // COUNT(*) per slot
  for (int j = 0; j < p.n_out; j++) {
    if (p.out_reg[j] == 255) continue;
    b += a4;                              // NULL arguments per slot
    if (ArgSum(p, j)) b += ns * 8 + a4;  // int64 sum + signed wrap count
    if (ArgMM(p, j)) b += ns * 16;
  }
  return b;
}

// The kernel: U rows per thread (hoisted loads, as the aggregate kernel),
// every selected row adds into a replica of its slot in LDS (lane % R picks
// the replica); sums are int64 in LDS with the rare signed wrap counted apart
// (exact int128 on merge).  One merge per block and slot at the end.
static std::string GroupSource(const VmProgram &p, const dev::VmCols &cols, const GroupSpec &g) {
  std::ostringstream o;
  const int nr = p.n_regs > 0 ? p.n_regs : 1;
  int U = 4;
  if (const char *e = Knob("MBX_JIT_GU")) U = atoi(e) == 1 || atoi(e) == 2 || atoi(e) == 8 ? atoi(e) : 4;
  o << kJitPrelude;
  o << "\nstruct LocalRF {\n  int64_t l[" << nr << "], h[" << nr << "];\n  uint8_t n[" << nr
    << "];\n  __device__ __forceinline__ int64_t &lo(int i) { return l[i]; }\n"
       "  __device__ __forceinline__ int64_t &hi(int i) { return h[i]; }\n"
       "  __device__ __forceinline__ uint8_t &nl(int i) { return n[i]; }\n};\n"
       "struct JAggState {\n  unsigned long long count, sum_lo;\n  long long sum_hi, min_i, max_i;\n  double sum_f;\n"
       "  unsigned long long min_f, max_f;\n};\n"
       "struct JGroup {\n  int64_t kmin[" << JIT_MAX_KEYS << "], radix[" << JIT_MAX_KEYS << "], stride[" << JIT_MAX_KEYS
    << "];\n  int32_t nslots, R;\n};\n";
  o << "extern \"C\" __global__ __launch_bounds__(256) void mbx_jit_group(mbx::VmProgram P, mbx::dev::VmCols C, "
       "int64_t nrows, int64_t rs, int64_t rstep, JGroup G, JAggState *states, unsigned long long *cstar, "
       "int32_t *err) {\n"
       "  using namespace mbx;\n  using namespace mbx::dev;\n  VmCols Cs = C;\n";
  Specialise(o, cols);
  // LDS slot tables (layout = GroupLdsBytes)
  o << "  extern __shared__ __attribute__((aligned(16))) unsigned char jlds[];\n"
       "  const int NS = G.nslots * G.R;\n  const size_t A4 = ((size_t)NS * 4 + 7) & ~(size_t)7;\n"
       "  unsigned char *lp = jlds;\n  unsigned int *cnt = (unsigned int *)lp;\n  lp += A4;\n";
  for (int j = 0; j < p.n_out; j++) {
    if (p.out_reg[j] == 255) continue;
    o << "  unsigned int *nul" << j << " = (unsigned int *)lp;\n  lp += A4;\n";
    if (ArgSum(p, j))
      o << "  long long *sum" << j << " = (long long *)lp;\n  lp += (size_t)NS * 8;\n  int *ovf" << j
        << " = (int *)lp;\n  lp += A4;\n";
    if (ArgMM(p, j))
      o << "  long long *mn" << j << " = (long long *)lp;\n  lp += (size_t)NS * 8;\n  long long *mx" << j
        << " = (long long *)lp;\n  lp += (size_t)NS * 8;\n";
  }
  o << "  for (int i = threadIdx.x; i < NS; i += blockDim.x) {\n    cnt[i] = 0;\n";
  for (int j = 0; j < p.n_out; j++) {
    if (p.out_reg[j] == 255) continue;
    o << "    nul" << j << "[i] = 0;\n";
    if (ArgSum(p, j)) o << "    sum" << j << "[i] = 0;\n    ovf" << j << "[i] = 0;\n";
    if (ArgMM(p, j)) o << "    mn" << j << "[i] = INT64_MAX;\n    mx" << j << "[i] = INT64_MIN;\n";
  }
  o << "  }\n  __syncthreads();\n  const int rep = (threadIdx.x & 63) % G.R;\n";
  o << "  const int64_t S = (int64_t)gridDim.x * blockDim.x;\n"
       "  for (int64_t base = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; base < nrows; base += " << U << " * S) {\n";
  for (int r = 0; r < U; r++)
    o << "    const int64_t row" << r << " = base + " << r << " * S;\n    const bool act" << r << " = row" << r
      << " < nrows;\n    const int64_t lrow" << r << " = act" << r << " ? row" << r << " : nrows - 1;\n    LocalRF R" << r
      << " = {};\n";
  for (int r = 0; r < U; r++) o << Preload(p, std::to_string(r), "lrow" + std::to_string(r), "act" + std::to_string(r));
  for (int r = 0; r < U; r++) {
    o << "    {\n      const int64_t lrow = lrow" << r << ";\n      const bool active = act" << r
      << ";\n      LocalRF &R = R" << r << ";\n";
    o << Body(p, std::to_string(r));
    o << "    }\n";
  }
  for (int r = 0; r < U; r++) {
    o << "    {\n      LocalRF &R = R" << r << ";\n      const bool sel = act" << r;
    if (p.pred_reg != 255) o << " && !R.nl(" << (int)p.pred_reg << ") && R.lo(" << (int)p.pred_reg << ") != 0";
    o << ";\n      if (sel) {\n        long long slot = 0;\n        bool okk = true;\n";
    for (int i = 0; i < g.nkeys; i++) {
      const int kr = g.key_reg[i];
      if (g.key_nullable[i])
        o << "        { const long long d = R.nl(" << kr << ") ? G.radix[" << i << "] - 1 : R.lo(" << kr << ") - G.kmin[" << i
          << "];\n          okk = okk && (unsigned long long)d < (unsigned long long)(R.nl(" << kr << ") ? G.radix[" << i
          << "] : G.radix[" << i << "] - 1);\n          slot += d * G.stride[" << i << "]; }\n";
      else
        o << "        { const long long d = R.lo(" << kr << ") - G.kmin[" << i << "];\n          okk = okk && !R.nl(" << kr
          << ") && (unsigned long long)d < (unsigned long long)G.radix[" << i << "];\n          slot += d * G.stride["
          << i << "]; }\n";
    }
    o << "        if (!okk) {\n          atomicCAS(err, 0, " << (int)E_KEY_RANGE << ");\n        } else {\n"
         "          const int sl = (int)slot * G.R + rep;\n          atomicAdd(&cnt[sl], 1u);\n";
    for (int j = 0; j < p.n_out; j++) {
      if (p.out_reg[j] == 255) continue;
      const int ar = p.out_reg[j];
      o << "          if (R.nl(" << ar << ")) {\n            atomicAdd(&nul" << j << "[sl], 1u);\n          } else {\n"
        << "            const long long v = R.lo(" << ar << ");\n";
      if (ArgSum(p, j))
        o << "            const long long old = (long long)atomicAdd((unsigned long long *)&sum" << j
          << "[sl], (unsigned long long)v);\n"
             "            const long long nw = (long long)((unsigned long long)old + (unsigned long long)v);\n"
             "            if (((old ^ nw) & (v ^ nw)) < 0) atomicAdd(&ovf" << j << "[sl], v < 0 ? -1 : 1);\n";
      if (ArgMM(p, j)) o << "            atomicMin(&mn" << j << "[sl], v);\n            atomicMax(&mx" << j << "[sl], v);\n";
      o << "          }\n";
    }
    o << "        }\n      }\n    }\n";
  }
  o << "  }\n  __syncthreads();\n"
       "  for (int q = threadIdx.x; q < G.nslots; q += blockDim.x) {\n"
       "    unsigned long long c = 0;\n    for (int r = 0; r < G.R; r++) c += cnt[q * G.R + r];\n"
       "    if (!c) continue;\n    atomicAdd(&cstar[q], c);\n";
  for (int j = 0; j < p.n_out; j++) {
    if (p.out_reg[j] == 255) continue;
    o << "    {\n      unsigned long long nn = 0, slo = 0;\n      long long shi = 0, a = INT64_MAX, b = INT64_MIN;\n"
         "      for (int r = 0; r < G.R; r++) {\n        const int sl = q * G.R + r;\n        nn += nul" << j << "[sl];\n";
    if (ArgSum(p, j))
      o << "        const long long v = sum" << j << "[sl];\n        const unsigned long long nlo = slo + (unsigned long long)v;\n"
           "        shi += (v >> 63) + (nlo < slo ? 1 : 0) + ovf" << j << "[sl];\n        slo = nlo;\n";
    if (ArgMM(p, j))
      o << "        a = mn" << j << "[sl] < a ? mn" << j << "[sl] : a;\n        b = mx" << j << "[sl] > b ? mx" << j
        << "[sl] : b;\n";
    o << "      }\n      const unsigned long long cj = c - nn;\n      if (cj) {\n"
         "        JAggState *st = states + (size_t)" << j << " * G.nslots + q;\n        atomicAdd(&st->count, cj);\n";
    if (ArgSum(p, j))
      o << "        const unsigned long long old = atomicAdd(&st->sum_lo, slo);\n"
           "        atomicAdd((unsigned long long *)&st->sum_hi, (unsigned long long)shi + ((old + slo) < old ? 1ull : 0ull));\n";
    if (ArgMM(p, j)) o << "        atomicMin(&st->min_i, a);\n        atomicMax(&st->max_i, b);\n";
    o << "      }\n    }\n";
  }
  o << "  }\n}\n";
  return o.str();
}

std::string GroupSourceForTest(const VmProgram &p, const dev::VmCols &cols, const GroupSpec &g) {
  return GroupSource(p, cols, g);
}

bool VmGroupAggregate(const VmProgram &p, const dev::VmCols &cols, const GroupSpec &g, int64_t nrows,
                      int64_t range_start, int64_t range_step, void *states, unsigned long long *count_star,
                      int32_t *err, hipStream_t s) {
  if (nrows <= 0 || g.nkeys < 1 || g.nkeys > JIT_MAX_KEYS || g.nslots < 1) return false;
  for (int j = 0; j < p.n_out; j++)
    if (p.out_reg[j] != 255 && p.out_class[j] != VC_I64) return false;
  // replicas: as many as fit 48 KiB (3 blocks per CU), at least one in 64 KiB
  int R = 64;
  if (const char *e = Knob("MBX_JIT_GR")) R = atoi(e) >= 1 && atoi(e) <= 64 ? atoi(e) : 64;
  while (R > 1 && GroupLdsBytes(p, g.nslots, R) > 48 * 1024) R >>= 1;
  const size_t lds = GroupLdsBytes(p, g.nslots, R);
  if (lds > 64 * 1024) return false;
  const std::string src = GroupSource(p, cols, g);
  hipFunction_t fn = GetNamed(src, "mbx_jit_group");
  if (!fn) return false;
  VmProgram P = p;
  dev::VmCols C = cols;
  JGroupArg G;
  memset(&G, 0, sizeof(G));
  for (int i = 0; i < g.nkeys; i++) {
    G.kmin[i] = g.kmin[i];
    G.radix[i] = g.radix[i];
    G.stride[i] = g.stride[i];
  }
  G.nslots = g.nslots;
  G.R = R;
  void *args[] = {&P, &C, &nrows, &range_start, &range_step, &G, &states, &count_star, &err};
  int cus = 0, d = 0;
  (void)hipGetDevice(&d);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, d);
  if (cus <= 0) cus = 256;
  int bpc = (int)std::min<size_t>(4, (160 * 1024) / std::max<size_t>(lds, 1));
  if (const char *e = Knob("MBX_JIT_GBPC")) bpc = atoi(e) >= 1 && atoi(e) <= 8 ? atoi(e) : bpc;
  if (bpc < 1) bpc = 1;
  int64_t gsz = (nrows + 1023) / 1024;
  if (gsz > (int64_t)cus * bpc) gsz = (int64_t)cus * bpc;
  return hipModuleLaunchKernel(fn, (unsigned)gsz, 1, 1, 256, 1, 1, (unsigned)lds, s, args, nullptr) == hipSuccess;
}

void JoinPending() { JoinAll(); }

bool VmAggregate(const VmProgram &p, const dev::VmCols &cols, int64_t nrows, int64_t range_start, int64_t range_step,
                 void *states, unsigned long long *count_star, int32_t *err, hipStream_t s) {
  if (nrows <= 0) return false;
  const std::string src = AggSource(p, cols);
  hipFunction_t fn = GetNamed(src, "mbx_jit_agg");
  if (!fn) return false;
  VmProgram P = p;
  dev::VmCols C = cols;
  void *args[] = {&P, &C, &nrows, &range_start, &range_step, &states, &count_star, &err};
  int cus = 0, d = 0;
  (void)hipGetDevice(&d);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, d);
  if (cus <= 0) cus = 256;
  // 4 blocks per CU (profiles/r01_jit_sweep.log: 0.384 ms vs 0.408 at 8)
  int bpc = 4;
  if (const char *e = Knob("MBX_JIT_BPC")) bpc = atoi(e) >= 1 && atoi(e) <= 32 ? atoi(e) : 4;
  int64_t g = (nrows + 255) / 256;
  if (g > (int64_t)cus * bpc) g = (int64_t)cus * bpc;
  return hipModuleLaunchKernel(fn, (unsigned)g, 1, 1, 256, 1, 1, 0, s, args, nullptr) == hipSuccess;
}

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
