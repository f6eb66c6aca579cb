// lbf_capi.cpp -- host side of liblbfhash.so: error slot, base64-27, device
// helpers and the lbf_ctx that streams host chunks through pinned staging to
// one or more MI355X devices.
//
// The context is the batched replacement for the reference's per-chunk
// fread -> Base64Encode loop (/root/reference/cpp/src/Encoder.cpp:54-72) and
// the per-chunk verify loops (Flood.cpp:246-285, ChunkMethods.cpp:111-128,
// 156-167): the caller hands over a descriptor table, the context copies the
// covered byte ranges into device slots (LBF_SLOTS of them, round-robin: host
// memcpy of group g+1 overlaps H2D + kernel + D2H of the groups before it) and
// returns digests or verdicts.
// Multiple devices take contiguous index ranges, one host thread each, with no
// collective.
#include <hip/hip_runtime.h>
#include <hsa/hsa_ext_amd.h>
#include <fcntl.h>
#include <pthread.h>
#include <sched.h>
#include <string.h>
#include <sys/resource.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <condition_variable>
#include <cerrno>
#include <cstdio>
#include <chrono>
#include <cstdlib>
#include <functional>
#include <iterator>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "lbf_internal.hpp"

namespace lbf {

namespace {
thread_local std::string t_last_error;
}

void set_error(const std::string& msg) { t_last_error = msg; }
const char* last_error_cstr() { return t_last_error.c_str(); }

int fail(int status, const std::string& msg) {
  set_error(msg);
  return status;
}

int hip_fail(hipError_t e, const char* what) {
  // HIP keeps a failed call's status as the thread's last error; left there,
  // it surfaces from the hipGetLastError() after the NEXT kernel launch and
  // fails a call that did nothing wrong.  The status is reported here instead.
  (void)hipGetLastError();
  return fail(e == hipErrorOutOfMemory ? LBF_ERR_NOMEM : LBF_ERR_HIP,
              std::string(what) + ": " + hipGetErrorString(e));
}

// Nothing is thrown across the C ABI: a host allocation that
// fails, or a thread that cannot be started, inside a call becomes a status.
template <class F>
int guarded(F&& f) {
  try {
    return f();
  } catch (const std::bad_alloc&) {
    return fail(LBF_ERR_NOMEM, "host allocation failed");
  } catch (const std::system_error& e) {
    return fail(LBF_ERR_NOMEM, std::string("host resources: ") + e.what());
  } catch (const std::exception& e) {
    return fail(LBF_ERR_INVALID, std::string("internal error: ") + e.what());
  }
}

}  // namespace lbf

using lbf::fail;
using lbf::guarded;
using lbf::hip_fail;

// ---------------------------------------------------------------------------
// base64-27 (BaseN_Encoder(alphabet, 6), no padding: basecode.cpp:13-37,39-104;
// alphabet Encoder.cpp:104-105).  20 bytes = 160 bits = 26 full sextets plus
// one 4-bit tail sextet, MSB first, zero-filled on the right.
// ---------------------------------------------------------------------------
static const char kAlphabet[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

extern "C" void lbf_b64_27(const uint8_t digest[20], char out[28]) {
  int o = 0;
  // 6 groups of 3 bytes -> 24 chars, then 2 bytes -> 3 chars (last one partial)
  for (int g = 0; g < 6; ++g) {
    const uint32_t v = (uint32_t(digest[3 * g]) << 16) | (uint32_t(digest[3 * g + 1]) << 8) | digest[3 * g + 2];
    out[o++] = kAlphabet[(v >> 18) & 63];
    out[o++] = kAlphabet[(v >> 12) & 63];
    out[o++] = kAlphabet[(v >> 6) & 63];
    out[o++] = kAlphabet[v & 63];
  }
  const uint32_t v = (uint32_t(digest[18]) << 8) | digest[19];  // 16 bits
  out[o++] = kAlphabet[(v >> 10) & 63];
  out[o++] = kAlphabet[(v >> 4) & 63];
  out[o++] = kAlphabet[(v << 2) & 63];
  out[o] = '\0';
}

static int b64_value(char c) {
  if (c >= 'A' && c <= 'Z') return c - 'A';
  if (c >= 'a' && c <= 'z') return c - 'a' + 26;
  if (c >= '0' && c <= '9') return c - '0' + 52;
  if (c == '+') return 62;
  if (c == '/') return 63;
  return -1;
}

extern "C" int lbf_b64_27_decode(const char* in, size_t len, uint8_t out[20]) {
  if (!in || !out || len != 27) return fail(LBF_ERR_INVALID, "b64_27_decode: need exactly 27 chars");
  uint32_t acc = 0;
  int bits = 0, o = 0;
  for (size_t i = 0; i < 27; ++i) {
    const int v = b64_value(in[i]);
    if (v < 0) return fail(LBF_ERR_INVALID, "b64_27_decode: character outside the alphabet");
    acc = (acc << 6) | (uint32_t)v;
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      if (o < 20) out[o++] = (uint8_t)(acc >> bits);
      acc &= (1u << bits) - 1u;
    }
  }
  // 162 bits read, 160 used: the 2 leftover bits must be zero (canonical form)
  if (o != 20 || bits != 2 || acc != 0) return fail(LBF_ERR_INVALID, "b64_27_decode: non-canonical tail");
  return LBF_OK;
}

// ---------------------------------------------------------------------------
// Library / device helpers
// ---------------------------------------------------------------------------
extern "C" int lbf_abi_version(void) { return LBF_ABI_VERSION; }

extern "C" const char* lbf_last_error(void) { return lbf::last_error_cstr(); }

extern "C" int lbf_device_count(int* out) {
  if (!out) return fail(LBF_ERR_INVALID, "null out");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *out = n;
  return LBF_OK;
}

extern "C" int lbf_dev_malloc(void** out, uint64_t bytes) {
  if (!out) return fail(LBF_ERR_INVALID, "null out");
  LBF_HIP_TRY(hipMalloc(out, bytes ? bytes : 1));
  return LBF_OK;
}
extern "C" int lbf_dev_free(void* p) {
  LBF_HIP_TRY(hipFree(p));
  return LBF_OK;
}
extern "C" int lbf_memcpy_h2d(void* dst, const void* src, uint64_t bytes) {
  LBF_HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
  return LBF_OK;
}
extern "C" int lbf_memcpy_d2h(void* dst, const void* src, uint64_t bytes) {
  LBF_HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
  return LBF_OK;
}
extern "C" int lbf_set_device(int d) {
  LBF_HIP_TRY(hipSetDevice(d));
  return LBF_OK;
}
extern "C" int lbf_device_synchronize(void) {
  LBF_HIP_TRY(hipDeviceSynchronize());
  return LBF_OK;
}
extern "C" int lbf_stream_create(void** out) {
  if (!out) return fail(LBF_ERR_INVALID, "null out");
  hipStream_t s;
  LBF_HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  *out = (void*)s;
  return LBF_OK;
}
extern "C" int lbf_stream_destroy(void* s) {
  LBF_HIP_TRY(hipStreamDestroy((hipStream_t)s));
  return LBF_OK;
}
extern "C" int lbf_stream_synchronize(void* s) {
  LBF_HIP_TRY(hipStreamSynchronize((hipStream_t)s));
  return LBF_OK;
}

// ---------------------------------------------------------------------------
// Context: workers (one per device, or LBF_WORKERS_PER_DEVICE per device for
// tests) with LBF_SLOTS pipeline slots each.
// ---------------------------------------------------------------------------
namespace {

uint64_t env_u64(const char* name, uint64_t dflt) {
  const char* v = getenv(name);
  if (!v || !*v) return dflt;
  return strtoull(v, nullptr, 10);
}

long env_long(const char* name, long dflt) {
  const char* v = getenv(name);
  if (!v || !*v) return dflt;
  return strtol(v, nullptr, 10);
}

// ---- NUMA placement -----------------------------
// Each worker's pinned staging is allocated on its GPU's NUMA node and its host
// threads (the worker thread of a multi-worker job and the staging-copy
// threads) run on that node's CPUs, so the host memcpy/pread writes local DRAM
// and the DMA engine reads it without crossing the socket link.  The node comes
// from the GPU's PCI bus id (/sys/bus/pci/devices/<id>/numa_node); LBF_NUMA=0
// turns placement off.  Raw syscalls: no libnuma dependency.
constexpr int kMpolDefault = 0, kMpolPreferred = 1;
constexpr unsigned long kMpolFNode = 1, kMpolFAddr = 2;
constexpr unsigned long kMaxNodes = 1024;

// The caller's current HIP device is its own state (a torch process keeps its
// tensors on it): entry points that switch devices to create, drive or free
// workers put it back on the way out.
struct KeepCurrentDevice {
  int saved = -1;
  KeepCurrentDevice() {
    if (hipGetDevice(&saved) != hipSuccess) saved = -1;
  }
  ~KeepCurrentDevice() {
    if (saved >= 0) (void)hipSetDevice(saved);
  }
};

bool numa_enabled() {
  static const bool on = env_long("LBF_NUMA", 1) != 0;
  return on;
}

std::string read_line(const std::string& path) {
  FILE* f = fopen(path.c_str(), "r");
  if (!f) return "";
  char buf[4096];
  std::string out;
  if (fgets(buf, sizeof(buf), f)) out = buf;
  fclose(f);
  while (!out.empty() && (out.back() == '\n' || out.back() == ' ')) out.pop_back();
  return out;
}

std::vector<int> parse_cpulist(const std::string& s) {  // "0-63,128-191"
  std::vector<int> out;
  size_t p = 0;
  while (p < s.size()) {
    char* end = nullptr;
    const long a = strtol(s.c_str() + p, &end, 10);
    if (end == s.c_str() + p) break;
    long b = a;
    p = (size_t)(end - s.c_str());
    if (p < s.size() && s[p] == '-') {
      b = strtol(s.c_str() + p + 1, &end, 10);
      p = (size_t)(end - s.c_str());
    }
    for (long c = a; c <= b && c < CPU_SETSIZE; ++c) out.push_back((int)c);
    if (p < s.size() && s[p] == ',') ++p;
    else break;
  }
  return out;
}

int device_numa_node(int device) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) return -1;
  std::string id(bus);
  for (char& c : id) c = (char)tolower((unsigned char)c);
  const std::string v = read_line("/sys/bus/pci/devices/" + id + "/numa_node");
  return v.empty() ? -1 : atoi(v.c_str());
}

// The node's CPUs that this process may run on (empty: no binding).
std::vector<int> node_cpus_allowed(int node) {
  if (node < 0) return {};
  const std::vector<int> cpus = parse_cpulist(read_line("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist"));
  cpu_set_t allowed;
  CPU_ZERO(&allowed);
  if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return {};
  std::vector<int> out;
  for (int c : cpus)
    if (CPU_ISSET(c, &allowed)) out.push_back(c);
  return out;
}

void bind_thread(const std::vector<int>& cpus) {
  if (cpus.empty()) return;
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int c : cpus) CPU_SET(c, &set);
  (void)pthread_setaffinity_np(pthread_self(), sizeof(set), &set);  // advisory: a refusal only costs locality
}

// MPOL_PREFERRED(node) for the calling thread while in scope.
struct PreferNode {
  bool active = false;
  int old_mode = kMpolDefault;
  unsigned long old_mask[kMaxNodes / 64] = {};
  explicit PreferNode(int node) {
    if (node < 0 || node >= (int)kMaxNodes) return;
    if (syscall(SYS_get_mempolicy, &old_mode, old_mask, kMaxNodes, nullptr, 0ul) != 0) return;
    unsigned long mask[kMaxNodes / 64] = {};
    mask[node / 64] = 1ul << (node % 64);
    active = syscall(SYS_set_mempolicy, kMpolPreferred, mask, kMaxNodes) == 0;
  }
  ~PreferNode() {
    if (!active) return;
    if (old_mode == kMpolDefault) (void)syscall(SYS_set_mempolicy, kMpolDefault, nullptr, 0ul);
    else (void)syscall(SYS_set_mempolicy, old_mode, old_mask, kMaxNodes);
  }
};

// NUMA node of the page holding `p` (-1 when unknown).
int page_node(const void* p) {
  if (!p) return -1;
  int node = -1;
  if (syscall(SYS_get_mempolicy, &node, nullptr, 0ul, const_cast<void*>(p), kMpolFNode | kMpolFAddr) != 0) return -1;
  return node;
}

// ---- workers and slots -----------------------------------------------------
// Staging is split in two rings.  A DEVICE slot in HBM holds one batch: the
// descriptors (offsets u64[cnt], sizes u32[cnt], expected 20 B x cnt, padded
// to kHdrAlign) and the chunk bytes, plus its stream and the batch's results;
// one kernel hashes the batch there and one D2H returns digests or verdicts.
// A HOST slot is a piece of pinned memory the batch's bytes pass through on
// their way to the device slot: a batch larger than a host slot is copied as
// several pieces (one H2D each) followed by its header, a batch that fits one
// host slot travels as one [header | data] copy.  A host slot is free again
// as soon as its H2D is done; a device slot only once its kernel is -- and
// that kernel lasts one chunk's serial SHA-1 chain (≈3.1 ms per 256 KiB of
// chunk, whatever the batch size).  So the device ring is sized per job to
// hold PCIe-rate x chain-time bytes in HBM (288 GB per GPU: the cheap place
// for bytes in flight), and the pinned ring stays small (LBF_SLOTS x
// LBF_PIN_MB): pinning is what a one-shot encode pays up front.
constexpr uint64_t kHdrAlign = 256;
constexpr uint64_t kDescBytes = 8 + 4 + 20;

uint64_t header_bytes(uint64_t cnt) { return (cnt * kDescBytes + kHdrAlign - 1) / kHdrAlign * kHdrAlign; }

struct HostSlot {
  uint8_t* h_buf = nullptr;      // pinned, pin_bytes
  hipEvent_t copied = nullptr;   // recorded after the H2D that last read h_buf
  bool in_flight = false;
};

struct DevSlot {
  hipStream_t stream = nullptr;
  uint8_t* d_buf = nullptr;  // header | data (hdr_cap + slot_bytes)
  uint8_t* h_hdr = nullptr;  // pinned header of a multi-piece batch (hdr_cap)
  uint8_t* h_edge = nullptr;  // pinned bounce for a direct batch's bytes outside the pinned pages (edge_cap())
  uint8_t* d_out = nullptr;  // desc_cap * 20: digests, or verdicts
  uint8_t* h_out = nullptr;  // pinned
  std::vector<uint8_t> ok;   // 1 = chunk bytes fully available
  hipEvent_t copied = nullptr;  // recorded after a direct-route batch's last H2D (see worker_run)
  // pending group (positions [g_begin, g_end)) to finalize after the stream drains
  bool pending = false;
  uint64_t g_begin = 0, g_end = 0;
};

// Helper threads of one worker's staging copies, started once and kept: a
// staging piece (LBF_PIN_MB, 128 MiB) moves in ≈2.5 ms at PCIe rate, and
// starting, binding and joining seven threads for every piece cost a
// measurable share of that.  run() hands the helpers a piece count and a
// function, joins in itself, and returns once every helper is done with it.
class CopyPool {
 public:
  CopyPool(unsigned helpers, const std::vector<int>& cpus) {
    for (unsigned t = 0; t < helpers; ++t) {
      try {
        th_.emplace_back([this, cpus] {
          bind_thread(cpus);
          loop();
        });
      } catch (const std::system_error&) {
        break;  // fewer helpers: the caller and the others take their pieces
      }
    }
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> lock(mu_);
      stop_ = true;
    }
    cv_work_.notify_all();
    for (std::thread& t : th_) t.join();
  }
  CopyPool(const CopyPool&) = delete;
  CopyPool& operator=(const CopyPool&) = delete;

  size_t helpers() const { return th_.size(); }

  // fn(q) for q in [0, n), spread over the caller and the helpers
  void run(size_t n, const std::function<void(size_t)>& fn) {
    {
      std::lock_guard<std::mutex> lock(mu_);
      fn_ = &fn;
      n_ = n;
      next_.store(0);
      busy_ = th_.size();
      ++gen_;
    }
    cv_work_.notify_all();
    pull(fn, n);
    std::unique_lock<std::mutex> lock(mu_);
    cv_done_.wait(lock, [this] { return busy_ == 0; });
    fn_ = nullptr;
  }

 private:
  void pull(const std::function<void(size_t)>& fn, size_t n) {
    for (size_t q; (q = next_++) < n;) fn(q);
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(size_t)>* fn;
      size_t n;
      {
        std::unique_lock<std::mutex> lock(mu_);
        cv_work_.wait(lock, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        fn = fn_;
        n = n_;
      }
      pull(*fn, n);
      std::lock_guard<std::mutex> lock(mu_);
      if (--busy_ == 0) cv_done_.notify_one();
    }
  }

  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_work_, cv_done_;
  const std::function<void(size_t)>* fn_ = nullptr;
  size_t n_ = 0;
  std::atomic<size_t> next_{0};
  size_t busy_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

struct Worker {
  int device = 0;
  int index = 0;            // position in the context
  int numa_node = -1;       // the device's NUMA node (-1: unknown / placement off)
  std::vector<int> cpus;    // CPUs its host threads bind to (empty: unbound)
  std::vector<HostSlot> host;  // LBF_SLOTS of them (default 3), used round-robin
  std::vector<DevSlot> dev;    // at least as many; grown per job for long chains, trimmed after it
  uint64_t slot_bytes = 0;  // current data capacity per device slot (grown on demand)
  uint64_t slot_max = 0;    // LBF_SLOT_MB: the largest a device slot may grow
  uint64_t pin_bytes = 0;   // current size of each pinned host slot (grown on demand)
  uint64_t pin_max = 0;     // LBF_PIN_MB: the largest a host slot may grow
  uint64_t dev_budget = 0;  // LBF_DEVICE_STAGING_MB: HBM for device slots
  uint64_t desc_cap = 0;    // descriptors per group
  uint64_t hdr_cap = 0;     // header_bytes(desc_cap)
  uint64_t bytes_staged = 0;  // chunk bytes sent through the pinned ring (cumulative)
  uint64_t bytes_direct = 0;  // chunk bytes sent straight from registered caller memory
  long fault_group = -1;    // LBF_TEST_FAULT_GROUP (tests only, one shot)
  bool fault_throws = false;  // LBF_TEST_FAULT_KIND=throw: the fault is a host exception, not a HIP error
  std::unique_ptr<CopyPool> pool;  // staging copy helpers, started by the first job that needs them
};

}  // namespace

namespace {
// Caller memory registered with lbf_host_register: [lo, hi) page-rounded, as
// pinned; `owned` = this context registered it (and unregisters it).
struct Registered {
  uintptr_t user = 0;  // the pointer the caller passed (the unregister key)
  uintptr_t user_end = 0;  // user + the length the caller passed
  uintptr_t lo = 0, hi = 0;
  bool owned = false;
};
}  // namespace

struct lbf_ctx {
  std::vector<Worker> workers;
  std::vector<Registered> regs;  // guarded by mu, like every job
  // lbf_b64_verify_batch's device memory (text, sextets, bytes, tables) on
  // worker 0's device: one allocation, grown on demand, guarded by mu
  uint8_t* b64_dev = nullptr;
  uint64_t b64_cap = 0;
  // lbf_b64_verify_batch's chunks by decode path (lbf_ctx_b64_stats), guarded by mu
  uint64_t b64_one_pass = 0, b64_general = 0;
  mutable std::mutex mu;
};

namespace {

// Pinned host memory on the worker's NUMA node (hipHostMallocNumaUser makes
// the allocation follow the calling thread's memory policy).  Allocations and
// frees of pinned memory pass one process-wide mutex.  The HIP runtime is
// thread-safe on its own; the mutex makes a context's teardown visibly happen
// before another context reuses the same pinned pages, which is what a
// ThreadSanitizer build (tools/tsan_build.sh) needs to see: it cannot look
// inside the uninstrumented runtime's allocator, and reported the reuse of a
// destroyed context's pages by the next one as a race.
std::mutex g_pinned_mu;

hipError_t host_alloc(const Worker& w, void** p, uint64_t bytes) {
  if (w.numa_node >= 0) {
    PreferNode pref(w.numa_node);
    if (pref.active) {
      std::lock_guard<std::mutex> lock(g_pinned_mu);
      return hipHostMalloc(p, bytes, hipHostMallocNumaUser);
    }
  }
  std::lock_guard<std::mutex> lock(g_pinned_mu);
  return hipHostMalloc(p, bytes, hipHostMallocDefault);
}

void host_free(void* p) {
  if (!p) return;
  std::lock_guard<std::mutex> lock(g_pinned_mu);
  (void)hipHostFree(p);  // release paths: a failure has nowhere to go
}

// An on-the-fly registration pins only the pages that lie wholly inside the
// job's bytes (pin_on_the_fly), so a direct batch may hold up to a page at
// each end of the job that is not pinned: those bytes are bounced through
// this much pinned memory per device slot.
uint64_t edge_cap() { return 2 * (uint64_t)sysconf(_SC_PAGESIZE); }

int dev_slot_init(Worker& w, DevSlot& d) {
  LBF_HIP_TRY(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
  LBF_HIP_TRY(hipMalloc((void**)&d.d_out, w.desc_cap * 20));
  LBF_HIP_TRY(host_alloc(w, (void**)&d.h_out, w.desc_cap * 20));
  LBF_HIP_TRY(host_alloc(w, (void**)&d.h_hdr, w.hdr_cap));
  LBF_HIP_TRY(host_alloc(w, (void**)&d.h_edge, edge_cap()));
  if (w.slot_bytes) LBF_HIP_TRY(hipMalloc((void**)&d.d_buf, w.hdr_cap + w.slot_bytes));
  LBF_HIP_TRY(hipEventCreateWithFlags(&d.copied, hipEventDisableTiming));
  d.ok.assign(w.desc_cap, 0);
  return LBF_OK;
}

void dev_slot_free(DevSlot& d) {
  // errors here have nowhere to go: the slot is being released
  if (d.stream) (void)hipStreamSynchronize(d.stream);
  if (d.d_buf) (void)hipFree(d.d_buf);
  if (d.d_out) (void)hipFree(d.d_out);
  host_free(d.h_out);
  host_free(d.h_hdr);
  host_free(d.h_edge);
  if (d.copied) (void)hipEventDestroy(d.copied);
  if (d.stream) (void)hipStreamDestroy(d.stream);
  d = DevSlot{};
}

// Staging memory is sized to the work, not reserved up front: pinning 2 x 512
// MiB costs ≈200 ms at context creation and ≈110 ms at destruction
// (tools/startup_probe.py), which a one-chunk Base64Encode or a small file
// should not pay.  Slots grow, never shrink, in 8 MiB steps up to slot_max.
constexpr uint64_t kSlotStep = 8ull << 20;

int ensure_slot_bytes(Worker& w, uint64_t need, uint64_t dev_cap) {
  auto round = [](uint64_t x, uint64_t cap) {
    return std::min(cap, (std::max(x, kSlotStep) + kSlotStep - 1) / kSlotStep * kSlotStep);
  };
  const uint64_t dev_need = round(need, dev_cap);
  const uint64_t pin_need = round(std::min(need, w.pin_max), w.pin_max);
  if (dev_need > w.slot_bytes) {
    for (DevSlot& d : w.dev) {
      LBF_HIP_TRY(hipStreamSynchronize(d.stream));
      if (d.d_buf) (void)hipFree(d.d_buf);
      d.d_buf = nullptr;
    }
    w.slot_bytes = 0;
    for (DevSlot& d : w.dev) LBF_HIP_TRY(hipMalloc((void**)&d.d_buf, w.hdr_cap + dev_need));
    w.slot_bytes = dev_need;
  }
  if (pin_need > w.pin_bytes) {
    for (DevSlot& d : w.dev) LBF_HIP_TRY(hipStreamSynchronize(d.stream));  // no H2D reads a host slot
    for (HostSlot& h : w.host) {
      host_free(h.h_buf);
      h.h_buf = nullptr;
      h.in_flight = false;
    }
    w.pin_bytes = 0;
    for (HostSlot& h : w.host) LBF_HIP_TRY(host_alloc(w, (void**)&h.h_buf, pin_need));
    w.pin_bytes = pin_need;
  }
  return LBF_OK;
}

// Device slots for a job whose longest staged chunk is `largest` bytes: enough
// to keep ≈50 GB/s of H2D going for one chain's duration (≈1 µs per 64-byte
// block, conservatively), never more than the process's hardware queues
// (GPU_MAX_HW_QUEUES, HIP's default 4): streams beyond that share a queue, and
// a batch's copies would then wait behind another slot's long kernel.  At
// least kDevSlots, at most the HBM budget.
constexpr uint64_t kDevSlots = 3;

int ensure_dev_slots(Worker& w, uint64_t largest, uint64_t groups) {
  static const uint64_t hw_queues = (uint64_t)std::max(2L, std::min(32L, env_long("GPU_MAX_HW_QUEUES", 4)));
  const double chain_us = ((double)largest / 64.0 + 2.0) * 1.0;
  const uint64_t in_flight = (uint64_t)(50e3 * chain_us);  // bytes at 50 GB/s
  const uint64_t per = w.hdr_cap + w.slot_bytes;
  uint64_t want = (in_flight + w.slot_bytes - 1) / std::max<uint64_t>(1, w.slot_bytes) + 1;
  want = std::min<uint64_t>(want, groups);
  want = std::min<uint64_t>(want, std::max<uint64_t>(1, w.dev_budget / per));
  want = std::min<uint64_t>(hw_queues, std::max<uint64_t>(want, std::min(kDevSlots, hw_queues)));
  while (w.dev.size() < want) {
    w.dev.emplace_back();
    if (int rc = dev_slot_init(w, w.dev.back())) {
      std::string msg = lbf_last_error();
      dev_slot_free(w.dev.back());
      w.dev.pop_back();
      if (w.dev.size() >= kDevSlots) break;  // fewer slots in flight: slower, not wrong
      return fail(rc, msg);
    }
  }
  return LBF_OK;
}

// After a job, give back the device slots beyond kDevSlots, and the HBM of
// batches grown past LBF_SLOT_MB for long chains (the next job sizes its own).
void trim_dev_slots(Worker& w) {
  while (w.dev.size() > kDevSlots) {
    dev_slot_free(w.dev.back());
    w.dev.pop_back();
  }
  if (w.slot_bytes > w.slot_max) {
    for (DevSlot& d : w.dev) {
      (void)hipStreamSynchronize(d.stream);  // drained already; errors were reported by the job
      if (d.d_buf) (void)hipFree(d.d_buf);
      d.d_buf = nullptr;
    }
    w.slot_bytes = 0;
  }
}

int worker_init(Worker& w, int device, int index) {
  w.device = device;
  w.index = index;
  w.slot_max = std::max<uint64_t>(env_u64("LBF_SLOT_MB", 512) << 20, 1ull << 20);
  w.pin_max = std::max<uint64_t>(env_u64("LBF_PIN_MB", 128) << 20, 1ull << 20);
  w.dev_budget = std::max<uint64_t>(env_u64("LBF_DEVICE_STAGING_MB", 16384) << 20, 1ull << 20);
  // Three pinned slots keep the PCIe link busy: with two, staging group g+2
  // waits for group g's H2D, so the link idles while the host copies.
  w.host.resize(std::min<uint64_t>(8, std::max<uint64_t>(2, env_u64("LBF_SLOTS", 3))));
  w.slot_bytes = 0;
  w.desc_cap = 1u << 16;
  w.hdr_cap = header_bytes(w.desc_cap);
  // Test hook: fail the g-th group this worker stages (once), after earlier
  // groups are in flight, to exercise the drain on the error path.
  if (env_long("LBF_TEST_FAULT_WORKER", 0) == index) w.fault_group = env_long("LBF_TEST_FAULT_GROUP", -1);
  const char* kind = getenv("LBF_TEST_FAULT_KIND");
  w.fault_throws = kind && strcmp(kind, "throw") == 0;
  LBF_HIP_TRY(hipSetDevice(device));
  if (numa_enabled()) {
    w.numa_node = device_numa_node(device);
    w.cpus = node_cpus_allowed(w.numa_node);
  }
  for (HostSlot& h : w.host) LBF_HIP_TRY(hipEventCreateWithFlags(&h.copied, hipEventDisableTiming));
  w.dev.resize(kDevSlots);
  for (DevSlot& d : w.dev)
    if (int rc = dev_slot_init(w, d)) return rc;
  return LBF_OK;
}

void worker_free(Worker& w) {
  w.pool.reset();  // idle between jobs: the helpers only need waking and joining
  if (hipSetDevice(w.device) != hipSuccess) return;
  // teardown: errors here have nowhere to go, the context is being destroyed
  for (DevSlot& d : w.dev) dev_slot_free(d);
  w.dev.clear();
  for (HostSlot& h : w.host) {
    host_free(h.h_buf);
    if (h.copied) (void)hipEventDestroy(h.copied);
    h = HostSlot{};
  }
}

// Host threads per staging copy: LBF_COPY_THREADS, default 8 (a GPU box's
// share of host cores is 16; two devices' workers may copy at once).
unsigned copy_threads() {
  static const unsigned n = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(64, env_u64("LBF_COPY_THREADS", 8)));
  return n;
}

// Where a job's bytes come from: caller memory (bounds-checked up front) or
// files read with pread (one descriptor table over several files: each
// descriptor names its file).  read_serial() returns the bytes available.
struct Source {
  const uint8_t* base = nullptr;  // memory source
  uint64_t base_len = 0;
  std::vector<int> fds;           // file source: one fd per file, -1 = could not be opened
  bool pinned = false;            // [base, base+base_len) lies in a lbf_host_register'ed range
  bool autopinned = false;        // ... or in the span run_job pinned for this job (pin_on_the_fly)
  // The pinned addresses of a pinned source, [pin_lo, pin_hi): all of it for
  // a registered one; for an on-the-fly one the pages wholly inside the job's
  // bytes, so up to a page at either end lies outside (bounced, worker_run).
  uintptr_t pin_lo = 0, pin_hi = 0;
  unsigned threads = copy_threads();  // staging copy threads

  bool from_files() const { return !fds.empty(); }
  bool exists(uint32_t file) const { return !from_files() || fds[file] >= 0; }

  uint64_t read_serial(uint8_t* dst, uint32_t file, uint64_t off, uint64_t len) const {
    if (!from_files()) {
      memcpy(dst, base + off, len);
      return len;
    }
    const int fd = fds[file];
    uint64_t got = 0;
    while (fd >= 0 && got < len) {
      const ssize_t r = pread(fd, dst + got, len - got, (off_t)(off + got));
      if (r <= 0) break;  // EOF or error: the rest is unavailable
      got += (uint64_t)r;
    }
    return got;
  }
};

// A run: consecutive descriptors whose byte ranges follow each other in the
// source, staged with one copy.  `dst` is its position in the slot's data
// area (same 16-byte phase as `src`); `avail` is how much of it was read.
struct Run {
  uint64_t src = 0, len = 0, dst = 0, avail = 0;
  uint32_t file = 0;
};

// Copy every run of a group into the slot's data area.  A single host thread
// copies ~17 GiB/s into pinned memory, a third of what PCIe Gen5 moves, so
// runs are cut into pieces of at most `step` bytes (≥ 8 MiB of work per
// thread; `step` rounded up to a page) that the caller and the worker's
// CopyPool helpers, bound to the staging's NUMA node, pull from a shared
// index: one long contiguous run
// and many small scattered ones copy in parallel alike.  (The ceil(total /
// parts) step must cover everything: rounding floor(len / parts) once left the
// last bytes of a range uncopied, tools/fuzz_gpu.py seed 23006099, pinned by
// test_staging_split_covers_tail.)
void read_runs(const Source& src, std::vector<Run>& runs, uint8_t* data, Worker& w) {
  constexpr uint64_t kMinPart = 8ull << 20;
  uint64_t total = 0;
  for (const Run& r : runs) total += r.len;
  const uint64_t parts = std::min<uint64_t>(src.threads, total / kMinPart);
  if (parts <= 1) {
    for (Run& r : runs) r.avail = src.read_serial(data + r.dst, r.file, r.src, r.len);
    return;
  }
  const uint64_t step = ((total + parts - 1) / parts + 4095) & ~4095ull;
  struct Piece {
    size_t run;
    uint64_t at, len, got;
  };
  std::vector<Piece> pieces;
  for (size_t k = 0; k < runs.size(); ++k)
    for (uint64_t a = 0; a < runs[k].len; a += step) pieces.push_back({k, a, std::min(step, runs[k].len - a), 0});
  const std::function<void(size_t)> copy = [&](size_t q) {
    Piece& pc = pieces[q];
    pc.got = src.read_serial(data + runs[pc.run].dst + pc.at, runs[pc.run].file, runs[pc.run].src + pc.at, pc.len);
  };
  static const bool use_pool = env_long("LBF_COPY_POOL", 1) != 0;  // 0: threads per call (A/B knob)
  if (use_pool) {
    // the worker's helpers (copy_threads() - 1 of them, bound to its node) plus
    // the calling thread, already bound by its worker
    if (!w.pool) w.pool.reset(new CopyPool(copy_threads() - 1, w.cpus));
    w.pool->run(pieces.size(), copy);
  } else {
    std::atomic<size_t> next{0};
    auto pull = [&] {
      for (size_t q; (q = next++) < pieces.size();) copy(q);
    };
    // parts - 1 helpers plus the calling thread; a helper that cannot be
    // started leaves its pieces to the others
    std::vector<std::thread> th;
    for (uint64_t t = 1; t < parts; ++t) {
      try {
        th.emplace_back([&] {
          bind_thread(w.cpus);
          pull();
        });
      } catch (const std::system_error&) {
        break;
      }
    }
    pull();
    for (auto& t : th) t.join();
  }
  // a run's readable prefix: its pieces in order up to the first short one
  std::vector<bool> short_seen(runs.size(), false);
  for (Run& r : runs) r.avail = 0;
  for (const Piece& pc : pieces) {
    if (short_seen[pc.run]) continue;
    runs[pc.run].avail += pc.got;
    if (pc.got < pc.len) short_seen[pc.run] = true;
  }
}

struct Job {
  Source src;
  const uint32_t* file_of = nullptr;  // file of each descriptor (null: all in file / buffer 0)
  const uint64_t* offsets;
  const uint32_t* sizes;
  const uint8_t* expected;  // null => hash mode
  uint8_t* digests;         // hash mode output
  uint8_t* verdicts;        // verify mode output
  uint32_t file(uint64_t k) const { return file_of ? file_of[k] : 0; }
};

// The order a worker stages its descriptors in: positions [begin, end) map to
// job indices through `perm` (empty = identity, the common sorted case).
struct Order {
  uint64_t begin = 0;
  std::vector<uint64_t> perm;
  uint64_t operator()(uint64_t pos) const { return perm.empty() ? pos : perm[pos - begin]; }
};

// Copy finished results of a slot's group (positions [g_begin, g_end)) to the
// caller's arrays.  Chunks that were not fully readable: verdict 0 (verify) or
// an LBF_ERR_IO (hash).
int finalize(const Job& job, const Order& order, DevSlot& s) {
  if (!s.pending) return LBF_OK;
  s.pending = false;
  const uint64_t cnt = s.g_end - s.g_begin;
  if (job.expected) {
    for (uint64_t k = 0; k < cnt; ++k) job.verdicts[order(s.g_begin + k)] = s.h_out[k] & s.ok[k];
    return LBF_OK;
  }
  for (uint64_t k = 0; k < cnt; ++k)
    if (!s.ok[k])
      return fail(LBF_ERR_IO, "chunk " + std::to_string(order(s.g_begin + k)) + " could not be read in full");
  if (order.perm.empty()) {
    memcpy(job.digests + 20 * s.g_begin, s.h_out, cnt * 20);
  } else {
    for (uint64_t k = 0; k < cnt; ++k) memcpy(job.digests + 20 * order(s.g_begin + k), s.h_out + 20 * k, 20);
  }
  return LBF_OK;
}

// One chunk that does not fit a slot: a dedicated device buffer, synchronous
// (device slot 0's stream and host slot 0's header, both idle by then).
int run_oversize(Worker& w, const Job& job, uint64_t i) {
  DevSlot& s = w.dev[0];
  HostSlot& h = w.host[0];
  LBF_HIP_TRY(hipStreamSynchronize(s.stream));
  const uint32_t sz = job.sizes[i];
  std::vector<uint8_t> host(sz ? sz : 1);
  std::vector<Run> one{Run{job.offsets[i], sz, 0, 0, job.file(i)}};
  read_runs(job.src, one, host.data(), w);
  const bool ok = one[0].avail == sz && job.src.exists(job.file(i));
  if (!ok) {
    if (job.expected) {
      job.verdicts[i] = 0;
      return LBF_OK;
    }
    return fail(LBF_ERR_IO, "chunk " + std::to_string(i) + " could not be read in full");
  }
  uint8_t* d = nullptr;
  LBF_HIP_TRY(hipMalloc((void**)&d, sz ? sz : 1));
  int rc = LBF_OK;
  do {
    // header of a one-chunk group: offset 0, size sz, expected digest
    const uint64_t off0 = 0;
    memcpy(h.h_buf, &off0, 8);
    memcpy(h.h_buf + 8, &sz, 4);
    if (job.expected) memcpy(h.h_buf + 12, job.expected + 20 * i, 20);
    if (hipMemcpy(d, host.data(), sz, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(s.d_buf, h.h_buf, kDescBytes, hipMemcpyHostToDevice) != hipSuccess) {
      rc = fail(LBF_ERR_HIP, "oversize chunk H2D failed");
      break;
    }
    const uint64_t* d_off = reinterpret_cast<const uint64_t*>(s.d_buf);
    const uint32_t* d_size = reinterpret_cast<const uint32_t*>(s.d_buf + 8);
    rc = lbf_sha1_launch(d, d_off, d_size, 1, job.expected ? nullptr : s.d_out, job.expected ? s.d_buf + 12 : nullptr,
                         job.expected ? s.d_out : nullptr, s.stream);
    if (rc) break;
    if (hipStreamSynchronize(s.stream) != hipSuccess) {
      rc = fail(LBF_ERR_HIP, "oversize kernel failed");
      break;
    }
    const hipError_t e = job.expected ? hipMemcpy(job.verdicts + i, s.d_out, 1, hipMemcpyDeviceToHost)
                                      : hipMemcpy(job.digests + 20 * i, s.d_out, 20, hipMemcpyDeviceToHost);
    if (e != hipSuccess) rc = fail(LBF_ERR_HIP, "oversize D2H failed");
  } while (0);
  (void)hipFree(d);
  return rc;
}

// Descriptors closer than this to the end of the current run join it: the gap
// is copied along (cheaper than another copy); the 16-byte padding between
// ReadVerifiedChunks' arena slots is the common case.
constexpr uint64_t kJoinGap = 4096;
// A registered (pinned) source goes to the device without the staging copy,
// one H2D per run, when its group's runs average at least kDirectMinRun:
// below that, per-copy overhead costs more than the host memcpy it saves.
// Measured on one MI355X (tools/e2e_sizes.py --register), with
// each batch's copies ordered after the previous batch's (worker_run): 14.4
// against 12.0-12.5 GiB/s staged at 64 MiB, 44.4-45.1 against 29.5-42.8 at
// 1 GiB, 49.6-50.6 against 33.6-49.5 at 4 GiB.  LBF_DIRECT_MAX_MB (an A/B
// knob) caps the job size that goes direct; by default every size does.
constexpr uint64_t kDirectMinRun = 1ull << 20;

// Pinning a large pageable job on the fly (opt-in with
// LBF_AUTOPIN=1: on by default in round 5, off since round 6).  A pageable job
// crosses host DRAM three times on the staged route (the caller's write, the
// staging memcpy's read and write, the DMA's read); a registered one once (§3).
// Round 5 timed hipHostRegister of a 4 GiB span at ~0.1 ms and turned this on,
// but that span had been registered before in the same process: on pages
// registered for the first time it costs 168-233 ms per 4 GiB of touched 4 KiB
// pages (the kind new[]/malloc give; 7.5 ms on transparent huge pages, ~700 ms
// on pages never touched), and only re-registering pages HIP has seen is cheap
// (tools/register_cost.py, profiles/r06/register_cost/).  So a job on a fresh
// 4 KiB-page buffer ran 3.6x slower pinned than staged at 4 GiB (294 against
// 81 ms) and 3.4x at 1 GiB, while a warm one gained 0-8 %.  A caller that hashes
// one buffer repeatedly registers it once (lbf_host_register); LBF_AUTOPIN=1
// pins each large job's pages for the job.  When on, run_job registers them in
// one piece before any worker starts and unregisters after every worker has
// drained; the workers see a registered source and take the direct route.  One
// registration per JOB, not per worker: the workers' index ranges meet inside
// a page unless the buffer is page-aligned, and two registrations of one page
// are refused below (round 5 first pinned per worker, and with two workers one
// of them staged).  A span HIP refuses to register is staged, and so is a
// batch whose copy HIP refuses (see worker_run).
//
// The pages pinned on the fly by running jobs, process-wide, [lo, hi) each.
// Two contexts hashing the same pageable buffer at once must not both register
// it (one's unregister could drop pages the other is still copying from), so a
// span that overlaps another job's, or a range pinned through
// lbf_host_register, is staged.  The other direction matters as much (ADVICE
// r05): lbf_host_register must never take a job's pages for "pinned by
// someone else" and adopt them, since the job unpins them when it ends; it
// waits on g_autopin_cv until no running job's pages overlap its range.  Lock
// order: a context's mu, then g_autopin_mu, then g_pin_mu.
bool pin_table_overlaps(uintptr_t lo, uintptr_t hi);  // lbf_host_register's table (below)
std::mutex g_autopin_mu;
std::condition_variable g_autopin_cv;       // notified when a span is released
std::map<uintptr_t, uintptr_t> g_autopin;  // lo -> hi of the spans reserved now
bool autopin_overlaps_locked(uintptr_t lo, uintptr_t hi) {
  auto next = g_autopin.lower_bound(lo);
  return (next != g_autopin.end() && next->first < hi) || (next != g_autopin.begin() && std::prev(next)->second > lo);
}
bool reserve_autopin(uintptr_t lo, uintptr_t hi) {
  std::lock_guard<std::mutex> g(g_autopin_mu);
  if (autopin_overlaps_locked(lo, hi) || pin_table_overlaps(lo, hi)) return false;
  g_autopin[lo] = hi;
  return true;
}
void release_autopin(uintptr_t lo) {
  {
    std::lock_guard<std::mutex> g(g_autopin_mu);
    g_autopin.erase(lo);
  }
  g_autopin_cv.notify_all();
}

// The pages wholly inside the job's bytes [lo, hi), registered for the life of
// the object (the owner destroys it only once every copy from them has
// landed).  Rounding inward, not outward, is what keeps the library off memory
// it was not handed: the first and last page of a span
// that does not start and end on a page boundary also hold the caller's other
// data, which the caller may pin itself while the job runs (an outward span
// made that hipHostRegister fail), so they stay pageable and a direct batch
// bounces the few bytes of the job that lie on them (worker_run).
class AutoPin {
 public:
  AutoPin(uintptr_t lo, uintptr_t hi) {
    const uintptr_t page = (uintptr_t)sysconf(_SC_PAGESIZE);
    lo_ = (lo + page - 1) & ~(page - 1);
    hi_ = hi & ~(page - 1);
    if (lo_ >= hi_ || !reserve_autopin(lo_, hi_)) return;  // another job pins (part of) it, or the caller does: staged
    reserved_ = true;
    const hipError_t e = hipHostRegister(reinterpret_cast<void*>(lo_), hi_ - lo_, hipHostRegisterPortable);
    if (e != hipSuccess) {
      (void)hipGetLastError();  // pinned elsewhere, or no memory: the job is staged
      return;
    }
    pinned_ = true;
  }
  ~AutoPin() {
    if (pinned_) {
      (void)hipHostUnregister(reinterpret_cast<void*>(lo_));
      (void)hipGetLastError();
    }
    if (reserved_) release_autopin(lo_);
  }
  AutoPin(const AutoPin&) = delete;
  AutoPin& operator=(const AutoPin&) = delete;
  bool pinned() const { return pinned_; }
  uintptr_t lo() const { return lo_; }
  uintptr_t hi() const { return hi_; }

 private:
  uintptr_t lo_ = 0, hi_ = 0;
  bool reserved_ = false, pinned_ = false;
};

// The registration run_job makes for a memory job of LBF_AUTOPIN_MIN_MB (64)
// and more whose chunks cover their address span without a gap, or null.  The
// union of the chunks is measured in offset order (a sorted copy of the table
// when it is not sorted already, so repeated chunks count once: ADVICE r05).
// A table with gaps is staged: pinning across a gap pins pages no copy reads,
// bytes the caller did not hand over (round 5 pinned any span its chunks
// filled half of).  A span larger than half of the host's physical memory is
// staged too: pinning it would lock most of RAM for the length of the call.
std::unique_ptr<AutoPin> pin_on_the_fly(const Job& job, uint64_t n) {
  if (job.src.from_files() || job.src.pinned || env_long("LBF_AUTOPIN", 0) != 1) return nullptr;
  const uint64_t min_bytes = env_u64("LBF_AUTOPIN_MIN_MB", 64) << 20;
  uint64_t lo = UINT64_MAX, hi = 0, sum = 0;
  bool sorted = true;
  for (uint64_t k = 0; k < n; ++k) {
    const uint64_t o = job.offsets[k], sz = job.sizes[k];
    if (sz == 0) continue;
    if (k && o < job.offsets[k - 1]) sorted = false;
    lo = std::min(lo, o);
    hi = std::max(hi, o + sz);
    sum += sz;
  }
  // the union is at most the sum and at most the span: both must reach the bar
  if (hi <= lo || hi - lo < min_bytes || sum < hi - lo) return nullptr;
  const long pages = sysconf(_SC_PHYS_PAGES), page = sysconf(_SC_PAGESIZE);
  if (pages > 0 && page > 0 && hi - lo > (uint64_t)pages * (uint64_t)page / 2) return nullptr;
  std::vector<uint64_t> perm;
  if (!sorted) {
    perm.resize(n);
    for (uint64_t k = 0; k < n; ++k) perm[k] = k;
    std::sort(perm.begin(), perm.end(), [&](uint64_t x, uint64_t y) { return job.offsets[x] < job.offsets[y]; });
  }
  uint64_t run_end = lo;
  for (uint64_t q = 0; q < n; ++q) {
    const uint64_t k = sorted ? q : perm[q], o = job.offsets[k], sz = job.sizes[k];
    if (sz == 0) continue;
    if (o > run_end) return nullptr;  // a gap
    run_end = std::max(run_end, o + sz);
  }
  const uintptr_t b = reinterpret_cast<uintptr_t>(job.src.base);
  std::unique_ptr<AutoPin> pin(new AutoPin(b + lo, b + hi));
  if (!pin->pinned()) pin.reset();
  return pin;
}

// Process descriptors [begin, end) on one worker.  They are staged in source
// order: sorted by offset (a stable permutation, skipped when the table is
// already sorted, as every file-order table is).  A group is a run of
// positions whose bytes fit a slot, packed as runs: a descriptor that starts
// inside, or within kJoinGap of, the current run extends it (a contiguous
// table is one run and one copy; overlapping chunks share their bytes); any
// other starts a new run at the next free position with its 16-byte phase.
// So a group holds as many chunks as their bytes fit, wherever they lie in
// the source.  (Round 1 grouped by the covering range of consecutive
// descriptors in caller order, which collapsed to one or two chunks per group
// for a scattered table: 8.5 s for 3,000 random chunks of a 160 MiB buffer,
// tools/staging_probe.py.)  One H2D per group, one kernel, one D2H; the host
// stages group g+1 while the GPU works on the groups before it.
//
// Every exit, error or not, passes the drain at the end: each slot's stream is
// synchronized and its pending group cleared, so nothing is still in flight
// and no stale group can be finalized into the next job's arrays.
int worker_run(Worker& w, const Job& job, uint64_t begin, uint64_t end) {
  LBF_HIP_TRY(hipSetDevice(w.device));
  Order order;
  order.begin = begin;
  auto before = [&](uint64_t x, uint64_t y) {  // source order: file, then offset
    const uint32_t fx = job.file(x), fy = job.file(y);
    return fx != fy ? fx < fy : job.offsets[x] < job.offsets[y];
  };
  for (uint64_t k = begin + 1; k < end; ++k)
    if (before(k, k - 1)) {
      order.perm.resize(end - begin);
      for (uint64_t q = begin; q < end; ++q) order.perm[q - begin] = q;
      std::stable_sort(order.perm.begin(), order.perm.end(), before);
      break;
    }
  uint64_t job_bytes = 0;  // the union of this worker's runs
  {
    // Staging sized to the bytes this worker stages (the union of its runs):
    // a quarter of them per slot once they exceed kSplitMin, so a mid-sized job
    // still runs as several groups whose copies, H2Ds and kernels overlap;
    // never below the largest chunk that fits a slot, and capped at slot_max.
    constexpr uint64_t kSplitMin = 32ull << 20;
    uint64_t bytes = 0, largest = 0, run_end = 0;
    uint32_t run_file = 0;
    bool open = false;
    for (uint64_t q = begin; q < end; ++q) {
      const uint64_t k = order(q), o = job.offsets[k], sz = job.sizes[k];
      if (sz == 0 || sz + 15 > w.slot_max) continue;
      largest = std::max(largest, sz);
      if (open && job.file(k) == run_file && o <= run_end + kJoinGap) {
        if (o + sz > run_end) bytes += o + sz - run_end, run_end = o + sz;
      } else {
        bytes += sz;
        run_end = o + sz;
        run_file = job.file(k);
        open = true;
      }
    }
    job_bytes = bytes;
    uint64_t per = bytes <= kSplitMin ? bytes : std::max({kSplitMin, (bytes + 3) / 4, largest});
    per = std::min(per, w.slot_max);
    // Long chains: a batch's kernel lasts one chain (≈1 µs per 64-byte block)
    // and at most ~4 batches are in flight (the hardware queues, see
    // ensure_dev_slots), so batches grow until three of them hold a chain's
    // worth of PCIe time -- beyond LBF_SLOT_MB, within a quarter of the HBM
    // budget and a quarter of the job.
    const uint64_t in_flight = (uint64_t)(50e3 * ((double)largest / 64.0 + 2.0));
    const uint64_t dev_cap = std::max(w.slot_max, w.dev_budget / 4);
    if (in_flight > 3 * per) per = std::max(per, std::min({in_flight / 3, dev_cap, (bytes + 3) / 4}));
    if (end > begin) {
      // (LBF_SLOT_MB stays the cap unless the long-chain rule raised the batch)
      if (int rc = ensure_slot_bytes(w, per + 16, per > w.slot_max ? dev_cap : w.slot_max)) return rc;
      const uint64_t groups = bytes / std::max<uint64_t>(1, w.slot_bytes) + 2;
      if (int rc = ensure_dev_slots(w, largest, groups)) return rc;
    }
  }
  // LBF_DIRECT_MAX_MB: A/B knob, the largest job (per worker) sent direct; unset = no limit
  const uint64_t direct_max_mb = env_u64("LBF_DIRECT_MAX_MB", 0);
  const uint64_t direct_max = direct_max_mb ? direct_max_mb << 20 : UINT64_MAX;
  const bool direct_job = job.src.pinned && job_bytes <= direct_max;
  int cur = 0, hcur = 0;
  int prev_direct = -1;  // device slot of the last direct-route batch
  uint64_t i = begin;
  int rc = LBF_OK;
  long group = 0;
  std::vector<Run> runs;
  std::vector<uint32_t> run_of;  // per position of the group: its run, or UINT32_MAX for an empty chunk
  auto hip_ok = [&rc](hipError_t e, const char* what) {
    if (e == hipSuccess) return true;
    rc = hip_fail(e, what);
    return false;
  };
  // An exception in the loop (a host allocation) must not skip the drain
  // below: groups may be in flight.
  try {
    while (i < end && rc == LBF_OK) {
      if ((uint64_t)job.sizes[order(i)] + 15 > w.slot_bytes) {
        for (DevSlot& s : w.dev) {
          if (!hip_ok(hipStreamSynchronize(s.stream), "hipStreamSynchronize")) break;
          if ((rc = finalize(job, order, s))) break;
        }
        if (rc == LBF_OK) rc = run_oversize(w, job, order(i));
        ++i;
        continue;
      }
      // group [i, j) of positions, packed as runs
      runs.clear();
      run_of.clear();
      uint64_t cursor = 0, j = i;
      while (j < end && j - i < w.desc_cap) {
        const uint64_t k = order(j), o = job.offsets[k], sz = job.sizes[k];
        if (sz == 0) {  // empty chunks take no bytes
          run_of.push_back(UINT32_MAX);
          ++j;
          continue;
        }
        if (sz + 15 > w.slot_bytes) break;  // oversize: the next group starts with it
        Run* r = runs.empty() ? nullptr : &runs.back();
        if (r && r->file == job.file(k) && o >= r->src && o <= r->src + r->len + kJoinGap) {
          const uint64_t new_len = std::max(r->len, o + sz - r->src);
          if (r->dst + new_len > w.slot_bytes) break;
          r->len = new_len;
          cursor = r->dst + new_len;
        } else {
          const uint64_t p = cursor + ((o - cursor) & 15u);
          if (p + sz > w.slot_bytes) break;
          runs.push_back(Run{o, sz, p, 0, job.file(k)});
          cursor = p + sz;
        }
        run_of.push_back((uint32_t)(runs.size() - 1));
        ++j;
      }
      DevSlot& s = w.dev[cur];
      if (!hip_ok(hipStreamSynchronize(s.stream), "hipStreamSynchronize")) break;
      if ((rc = finalize(job, order, s))) break;
      if (group++ == w.fault_group) {
        w.fault_group = -1;
        if (w.fault_throws) throw std::bad_alloc();  // must still reach the drain
        rc = fail(LBF_ERR_HIP, "injected fault (LBF_TEST_FAULT_GROUP) at group " + std::to_string(group - 1));
        break;
      }
      const uint64_t cnt = j - i;
      const uint64_t hdr = header_bytes(cnt);
      // The batch's bytes, [0, cursor) of its data area, go through the host
      // ring: in one [header | data] copy when they fit a host slot, else in
      // pieces of pin_bytes followed by the header from the slot's own pinned
      // header buffer.  A run cut by a piece boundary is read in parts; once a
      // part comes back short (EOF), the rest of that run is unavailable.
      // A registered source skips the ring: each run is copied to the device
      // straight from the caller's pinned memory, then the header follows.
      bool direct = direct_job && !runs.empty() && cursor >= runs.size() * kDirectMinRun;
      uint64_t edge_bytes = 0;
      for (Run& r : runs) r.avail = 0;
      if (direct) {
        // A batch's copies start only once the previous direct batch's have
        // landed.  Issued freely, the copies of every batch in the ring shared
        // the link, all batches finished copying together, and the link then
        // sat idle through their kernels (rocprofv3 trace,
        // profiles/r02/registered_trace/direct_ordered/).  In order, batch g
        // is hashed while batch g+1 is still copying, as on the staged route.
        if (prev_direct >= 0 && prev_direct != cur &&
            !hip_ok(hipStreamWaitEvent(s.stream, w.dev[prev_direct].copied, 0), "hipStreamWaitEvent"))
          break;
        // One copy per run (LBF_DIRECT_PIECE_MB, an A/B knob, cuts runs into pieces of that
        // size).  Before the copies were ordered, 32 MiB pieces helped (4 GiB 42.5 -> 47.2
        // GiB/s, profiles/r02/registered_trace/piece_sweep/); ordered, whole runs are as fast
        // or faster (50.6 against 49.6-49.8 GiB/s at 4 GiB, direct_ordered/).
        const uint64_t piece = env_u64("LBF_DIRECT_PIECE_MB", 0) << 20;
        bool refused = false;  // a copy HIP refuses from an on-the-fly registration (see below)
        // A run's bytes outside the pinned pages (an on-the-fly span's first
        // and last partial page, AutoPin) go through the slot's pinned bounce:
        // the slot's stream is idle here, so its previous contents are spent.
        // Bytes that do not fit it send the batch through staging.
        const uint64_t pin_lo = job.src.pin_lo - reinterpret_cast<uintptr_t>(job.src.base);
        const uint64_t pin_hi = job.src.pin_hi - reinterpret_cast<uintptr_t>(job.src.base);
        uint64_t bounced = 0;
        auto copy = [&](uint64_t dst, uint64_t src, uint64_t len) {  // one H2D of source bytes [src, src + len)
          const uint8_t* from = job.src.base + src;
          if (src < pin_lo || src + len > pin_hi) {
            if (bounced + len > edge_cap()) {
              refused = true;
              return;
            }
            memcpy(s.h_edge + bounced, from, len);
            from = s.h_edge + bounced;
            bounced += len;
          }
          const hipError_t e = hipMemcpyAsync(s.d_buf + w.hdr_cap + dst, from, len, hipMemcpyHostToDevice, s.stream);
          if (e == hipErrorInvalidValue && job.src.autopinned) {
            // HIP lets a span be registered over a range the caller had
            // pinned itself, then resolves copies in that range to the
            // caller's (smaller) registration and refuses them at enqueue.
            // Such a batch is staged; the copies already queued run before
            // the staged ones on the same stream, which overwrite whatever
            // they wrote.
            (void)hipGetLastError();
            refused = true;
          } else {
            hip_ok(e, "hipMemcpyAsync(H2D, registered source)");
          }
        };
        for (Run& r : runs) {
          // [r.src, r.src + r.len) cut at the pinned pages' ends: head, body, tail
          const uint64_t end = r.src + r.len;
          const uint64_t b0 = std::min(std::max(r.src, pin_lo), end), b1 = std::max(std::min(end, pin_hi), b0);
          if (b0 > r.src) copy(r.dst, r.src, b0 - r.src);
          const uint64_t step = piece ? piece : b1 - b0;
          for (uint64_t at = b0, len = 0; at < b1 && rc == LBF_OK && !refused; at += len) {
            len = std::min(step, b1 - at);
            copy(r.dst + (at - r.src), at, len);
          }
          if (end > b1 && rc == LBF_OK && !refused) copy(r.dst + (b1 - r.src), b1, end - b1);
          if (rc || refused) break;
          r.avail = r.len;
        }
        edge_bytes = refused ? 0 : bounced;
        if (rc) break;
        if (refused) {
          direct = false;
          for (Run& r : runs) r.avail = 0;
        } else {
          if (!hip_ok(hipEventRecord(s.copied, s.stream), "hipEventRecord")) break;
          prev_direct = cur;
        }
      }
      const bool single = !direct && hdr + cursor <= w.pin_bytes;
      const uint64_t data_off = single ? hdr : w.hdr_cap;
      uint8_t* h_header = nullptr;
      // (a direct batch's bounced edge bytes count as staged: they took a host copy)
      (direct ? w.bytes_direct : w.bytes_staged) += cursor - edge_bytes;
      w.bytes_staged += edge_bytes;
      std::vector<bool> cut_short(runs.size(), false);
      size_t first_run = 0;
      for (uint64_t pstart = 0; !direct && (pstart < cursor || (single && pstart == 0)) && rc == LBF_OK;) {
        const uint64_t room = single ? cursor : w.pin_bytes;
        const uint64_t pend = std::min(cursor, pstart + room);
        HostSlot& h = w.host[hcur];
        if (h.in_flight && !hip_ok(hipEventSynchronize(h.copied), "hipEventSynchronize")) break;  // its last H2D is done
        h.in_flight = false;
        uint8_t* piece = h.h_buf + (single ? hdr : 0);
        std::vector<Run> parts;
        std::vector<size_t> part_of;
        while (first_run < runs.size() && runs[first_run].dst + runs[first_run].len <= pstart) ++first_run;
        for (size_t r = first_run; r < runs.size() && runs[r].dst < pend; ++r) {
          const uint64_t a0 = std::max(runs[r].dst, pstart), a1 = std::min(runs[r].dst + runs[r].len, pend);
          if (a1 <= a0 || cut_short[r]) continue;
          parts.push_back(Run{runs[r].src + (a0 - runs[r].dst), a1 - a0, a0 - pstart, 0, runs[r].file});
          part_of.push_back(r);
        }
        read_runs(job.src, parts, piece, w);
        for (size_t q = 0; q < parts.size(); ++q) {
          Run& r = runs[part_of[q]];
          r.avail += parts[q].avail;
          if (parts[q].avail < parts[q].len) cut_short[part_of[q]] = true;
        }
        if (single) {
          h_header = h.h_buf;  // the header is written below, then header + data go in one copy
          break;
        }
        if (!hip_ok(hipMemcpyAsync(s.d_buf + data_off + pstart, piece, pend - pstart, hipMemcpyHostToDevice, s.stream),
                    "hipMemcpyAsync(H2D)") ||
            !hip_ok(hipEventRecord(h.copied, s.stream), "hipEventRecord"))
          break;
        h.in_flight = true;
        hcur = (hcur + 1) % (int)w.host.size();
        pstart = pend;
      }
      if (rc) break;
      if (!single) h_header = s.h_hdr;
      uint64_t* h_off = reinterpret_cast<uint64_t*>(h_header);
      uint32_t* h_size = reinterpret_cast<uint32_t*>(h_header + 8 * cnt);
      uint8_t* h_exp = h_header + 12 * cnt;
      for (uint64_t q = 0; q < cnt; ++q) {
        const uint64_t k = order(i + q), o = job.offsets[k], sz = job.sizes[k];
        const uint32_t r = run_of[q];
        // An empty chunk of an existing file is always readable, wherever it
        // lies: the reference's fseek succeeds past EOF and fread of 0 bytes
        // returns 0 (Flood.cpp:259-275); a file that cannot be opened leaves every
        // chunk '0' (Flood.cpp:257).  Unreadable chunks must not be hashed from
        // stale slot bytes: they get size 0 on the device (result discarded).
        s.ok[q] = (r == UINT32_MAX ? job.src.exists(job.file(k)) : o + sz <= runs[r].src + runs[r].avail) ? 1 : 0;
        h_off[q] = (r != UINT32_MAX && s.ok[q]) ? runs[r].dst + (o - runs[r].src) : 0;
        h_size[q] = s.ok[q] ? (uint32_t)sz : 0;
        if (job.expected) memcpy(h_exp + 20 * q, job.expected + 20 * k, 20);
      }
      {
        // header (+ data, for a single-piece batch) after the pieces, on the same stream
        HostSlot& h = w.host[hcur];
        const uint64_t bytes = single ? hdr + cursor : hdr;
        if (!hip_ok(hipMemcpyAsync(s.d_buf, h_header, bytes, hipMemcpyHostToDevice, s.stream), "hipMemcpyAsync(H2D)"))
          break;
        if (single) {
          if (!hip_ok(hipEventRecord(h.copied, s.stream), "hipEventRecord")) break;
          h.in_flight = true;
          hcur = (hcur + 1) % (int)w.host.size();
        }
      }
      const uint64_t* d_off = reinterpret_cast<const uint64_t*>(s.d_buf);
      const uint32_t* d_size = reinterpret_cast<const uint32_t*>(s.d_buf + 8 * cnt);
      if (job.expected)
        rc = lbf_sha1_launch(s.d_buf + data_off, d_off, d_size, cnt, nullptr, s.d_buf + 12 * cnt, s.d_out, s.stream);
      else rc = lbf_sha1_launch(s.d_buf + data_off, d_off, d_size, cnt, s.d_out, nullptr, nullptr, s.stream);
      if (rc) break;
      if (!hip_ok(hipMemcpyAsync(s.h_out, s.d_out, cnt * (job.expected ? 1 : 20), hipMemcpyDeviceToHost, s.stream),
                  "hipMemcpyAsync(D2H)"))
        break;
      s.pending = true;
      s.g_begin = i;
      s.g_end = j;
      cur = (cur + 1) % (int)w.dev.size();
      i = j;
    }
  } catch (const std::bad_alloc&) {
    rc = fail(LBF_ERR_NOMEM, "host allocation failed while staging");
  } catch (const std::system_error& e) {
    rc = fail(LBF_ERR_NOMEM, std::string("host resources while staging: ") + e.what());
  } catch (const std::exception& e) {
    rc = fail(LBF_ERR_INVALID, std::string("internal error while staging: ") + e.what());
  }
  // drain, on every path (every H2D ran on a device slot's stream, so this also
  // completes every host slot's copy)
  for (DevSlot& s : w.dev) {
    const hipError_t e = hipStreamSynchronize(s.stream);
    if (e != hipSuccess && rc == LBF_OK) rc = hip_fail(e, "hipStreamSynchronize");
    if (rc == LBF_OK) rc = finalize(job, order, s);
    s.pending = false;
  }
  for (HostSlot& h : w.host) h.in_flight = false;
  trim_dev_slots(w);
  return rc;
}

int validate_memory_job(const Job& job, uint64_t n) {
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t o = job.offsets[i], sz = job.sizes[i];
    if (o > job.src.base_len || sz > job.src.base_len - o)
      return fail(LBF_ERR_INVALID, "chunk " + std::to_string(i) + " lies outside [base, base+base_len)");
  }
  return LBF_OK;
}

// Contiguous index ranges per worker, one host thread each (bound to its
// worker's NUMA node), no collective.
// A memory source lies in a registered range: the pages this library pinned,
// or, for memory pinned by someone else, the caller's own bytes (only those
// were shown to lie in one pinned allocation, lbf_host_register).
bool in_registered(const lbf_ctx* ctx, const uint8_t* base, uint64_t len) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(base);
  for (const Registered& r : ctx->regs) {
    const uintptr_t lo = r.owned ? r.lo : r.user, hi = r.owned ? r.hi : r.user_end;
    if (a >= lo && a <= hi && len <= hi - a) return true;
  }
  return false;
}

int run_job(lbf_ctx* ctx, Job job, uint64_t n) {
  std::lock_guard<std::mutex> lock(ctx->mu);
  KeepCurrentDevice keep;  // worker 0 (and any inline worker) runs on this thread
  if (!job.src.from_files() && in_registered(ctx, job.src.base, job.src.base_len)) {
    job.src.pinned = true;
    job.src.pin_lo = reinterpret_cast<uintptr_t>(job.src.base);
    job.src.pin_hi = job.src.pin_lo + job.src.base_len;
  }
  // Declared before the workers run and destroyed after they return: every
  // worker drains its streams before returning, so no copy outlives the span.
  const std::unique_ptr<AutoPin> autopin = pin_on_the_fly(job, n);
  if (autopin) {
    job.src.pinned = job.src.autopinned = true;
    job.src.pin_lo = autopin->lo();
    job.src.pin_hi = autopin->hi();
  }
  if (const uint64_t hold = env_u64("LBF_TEST_AUTOPIN_HOLD_MS", 0); hold && autopin)
    std::this_thread::sleep_for(std::chrono::milliseconds(hold));  // tests only: keep the span pinned a while
  const size_t nw = ctx->workers.size();
  if (nw == 1 || n < 2 * nw) return worker_run(ctx->workers[0], job, 0, n);
  std::vector<int> rcs(nw, LBF_OK);
  std::vector<std::string> errs(nw);
  std::vector<std::thread> th;
  auto part = [&](size_t d, bool bind) {
    if (bind) bind_thread(ctx->workers[d].cpus);
    rcs[d] = guarded([&] { return worker_run(ctx->workers[d], job, n * d / nw, n * (d + 1) / nw); });
    if (rcs[d]) errs[d] = lbf_last_error();
  };
  std::vector<size_t> inline_parts;  // workers whose thread could not be started run here, in turn
  for (size_t d = 0; d < nw; ++d) {
    try {
      th.emplace_back(part, d, true);
    } catch (const std::system_error&) {
      inline_parts.push_back(d);
    }
  }
  for (size_t d : inline_parts) part(d, false);
  for (auto& t : th) t.join();
  for (size_t d = 0; d < nw; ++d)
    if (rcs[d])
      return fail(rcs[d], "worker " + std::to_string(d) + " (device " + std::to_string(ctx->workers[d].device) +
                              "): " + errs[d]);
  return LBF_OK;
}

// Device-pointer batch: synchronous on worker 0's first stream.
int run_device_job(lbf_ctx* ctx, const uint8_t* base, const uint64_t* offsets, const uint32_t* sizes,
                   uint64_t n, uint8_t* digests, const uint8_t* expected, uint8_t* verdicts) {
  std::lock_guard<std::mutex> lock(ctx->mu);
  KeepCurrentDevice keep;
  Worker& w = ctx->workers[0];
  LBF_HIP_TRY(hipSetDevice(w.device));
  hipStream_t s = w.dev[0].stream;
  for (uint64_t i = 0; i < n; i += 0xFFFFFFFFull) {
    const uint64_t cnt = std::min<uint64_t>(n - i, 0xFFFFFFFFull);
    int rc = lbf_sha1_launch(base, offsets + i, sizes + i, cnt, digests ? digests + 20 * i : nullptr,
                             expected ? expected + 20 * i : nullptr, verdicts ? verdicts + i : nullptr, s);
    if (rc) return rc;
  }
  LBF_HIP_TRY(hipStreamSynchronize(s));
  return LBF_OK;
}

}  // namespace

// Caller-pinned sources (lbf_host_register).  hipHostRegister pins whole
// pages, portably (every device can DMA from them).  HIP does not count
// registrations per caller: when a second context registered and then
// unregistered a range the first one held, the first one's pin was gone
// (its hipHostUnregister then failed; tests/test_gpu_registered.py, first
// run).  So the library keeps one process-wide pin table: contexts
// registering the same range share one pin (reference-counted), and memory
// that something else already pinned (a hipHostMalloc'd buffer, a caller's
// own hipHostRegister) is used as it is and never unpinned here.
namespace {
struct Pin {
  uintptr_t hi = 0;
  uint64_t refs = 0;
};
std::mutex g_pin_mu;
std::map<uintptr_t, Pin> g_pins;  // lo -> pin, disjoint ranges

bool pin_table_overlaps(uintptr_t lo, uintptr_t hi) {
  std::lock_guard<std::mutex> g(g_pin_mu);
  auto next = g_pins.lower_bound(lo);
  return (next != g_pins.end() && next->first < hi) || (next != g_pins.begin() && std::prev(next)->second.hi > lo);
}

// The pinned host allocation that holds address p, as [base, end), if any.
// hipMemGetAddressRange resolves host-pinned memory (hipHostMalloc,
// hipHostRegister) by the host address or, failing that, by the device
// address hipPointerGetAttributes reports for it.
struct PinnedAlloc {
  bool pinned = false;
  uintptr_t base = 0, end = 0;  // end == 0: the extent is unknown
  uint64_t id = 0;              // HIP's buffer id of the allocation (0: unknown)
};
PinnedAlloc pinned_alloc(uintptr_t p) {
  PinnedAlloc out;
  // The runtime under HIP reports the host base and size of the allocation a
  // pinned pointer lies in, for hipHostMalloc (an HSA pool allocation) and for
  // hipHostRegister (locked) memory alike.  hipMemGetAddressRange gives the
  // size of a hipHostRegister'd range but a null base (measured on the box,
  // tools/pin_extent_probe.py), so it is only the fallback.
  hsa_amd_pointer_info_t info{};
  info.size = sizeof(info);
  if (hsa_amd_pointer_info(reinterpret_cast<const void*>(p), &info, nullptr, nullptr, nullptr) == HSA_STATUS_SUCCESS &&
      (info.type == HSA_EXT_POINTER_TYPE_LOCKED || info.type == HSA_EXT_POINTER_TYPE_HSA) && info.hostBaseAddress &&
      info.sizeInBytes) {
    const uintptr_t b = reinterpret_cast<uintptr_t>(info.hostBaseAddress);
    if (b <= p && p - b < info.sizeInBytes) {
      out.pinned = true;
      out.base = b;
      out.end = b + info.sizeInBytes;
      return out;
    }
  }
  hipPointerAttribute_t attr{};
  out.pinned = hipPointerGetAttributes(&attr, reinterpret_cast<void*>(p)) == hipSuccess &&
               attr.type == hipMemoryTypeHost;
  (void)hipGetLastError();  // pageable memory is an error to that query
  if (!out.pinned) return out;
  // One id per allocation or registration: two addresses with the same id lie
  // in one allocation, and so does every byte between them.
  unsigned long long id = 0;
  if (hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, reinterpret_cast<hipDeviceptr_t>(p)) == hipSuccess)
    out.id = id;
  (void)hipGetLastError();
  const uintptr_t dev = reinterpret_cast<uintptr_t>(attr.devicePointer);
  for (const uintptr_t q : {p, dev}) {
    hipDeviceptr_t b = nullptr;
    size_t size = 0;
    const bool ok = q && hipMemGetAddressRange(&b, &size, reinterpret_cast<hipDeviceptr_t>(q)) == hipSuccess;
    (void)hipGetLastError();
    const uintptr_t bb = reinterpret_cast<uintptr_t>(b);
    if (ok && size && bb <= q && q - bb < size) {
      out.base = p - (q - bb);  // the same offset from the host base
      out.end = out.base + size;
      return out;
    }
  }
  return out;
}

// Drop one reference to the pin at lo (pinned by this library).
int unpin(uintptr_t lo) {
  std::lock_guard<std::mutex> lock(g_pin_mu);
  auto it = g_pins.find(lo);
  if (it == g_pins.end()) return LBF_OK;
  if (--it->second.refs) return LBF_OK;
  g_pins.erase(it);
  LBF_HIP_TRY(hipHostUnregister(reinterpret_cast<void*>(lo)));
  return LBF_OK;
}
}  // namespace

extern "C" int lbf_ctx_create(uint32_t device_mask, lbf_ctx** out) {
  if (!out) return fail(LBF_ERR_INVALID, "null out");
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return fail(LBF_ERR_NO_DEVICE, "no GPU visible: the chunk-hash path runs only on MI355X (no CPU fallback)");
  // Test knob: k workers per selected device, so the multi-worker split, the
  // per-worker staging and the error propagation of run_job run on a one-GPU
  // box exactly as they do with one worker per GPU on an 8-GPU node.
  const int per_dev = (int)std::max(1L, std::min(16L, env_long("LBF_WORKERS_PER_DEVICE", 1)));
  KeepCurrentDevice keep;  // worker_init selects each worker's device
  lbf_ctx* ctx = new (std::nothrow) lbf_ctx();
  if (!ctx) return fail(LBF_ERR_NOMEM, "host allocation failed");
  const int rc = guarded([&] {
    ctx->workers.reserve((size_t)std::min(ndev, 32) * (size_t)per_dev);  // workers never move once initialised
    for (int d = 0; d < ndev && d < 32; ++d) {
      if (device_mask && !(device_mask & (1u << d))) continue;
      for (int k = 0; k < per_dev; ++k) {
        ctx->workers.emplace_back();
        if (int r = worker_init(ctx->workers.back(), d, (int)ctx->workers.size() - 1)) return r;
      }
    }
    return (int)LBF_OK;
  });
  if (rc) {
    std::string msg = lbf_last_error();
    lbf_ctx_destroy(ctx);
    return fail(rc, msg);
  }
  if (ctx->workers.empty()) {
    delete ctx;
    return fail(LBF_ERR_NO_DEVICE, "device_mask selects no visible device");
  }
  *out = ctx;
  return LBF_OK;
}

extern "C" int lbf_ctx_worker_info(const lbf_ctx* ctx, int worker, int* device, int* numa_node, int* staging_node,
                                   int* bound_cpus) {
  if (!ctx || worker < 0 || worker >= (int)ctx->workers.size()) return fail(LBF_ERR_INVALID, "no such worker");
  // a running job may grow or trim the slots read below: wait for it
  std::lock_guard<std::mutex> lock(ctx->mu);
  const Worker& w = ctx->workers[worker];
  if (device) *device = w.device;
  if (numa_node) *numa_node = w.numa_node;
  if (staging_node)
    *staging_node = page_node(!w.host.empty() && w.host[0].h_buf ? (const void*)w.host[0].h_buf
                                                                 : (w.dev.empty() ? nullptr : (const void*)w.dev[0].h_out));
  if (bound_cpus) *bound_cpus = (int)w.cpus.size();
  return LBF_OK;
}

extern "C" void lbf_ctx_destroy(lbf_ctx* ctx) {
  if (!ctx) return;
  KeepCurrentDevice keep;
  if (ctx->b64_dev && !ctx->workers.empty() && hipSetDevice(ctx->workers[0].device) == hipSuccess)
    (void)hipFree(ctx->b64_dev);
  for (Worker& w : ctx->workers) worker_free(w);
  for (const Registered& r : ctx->regs)
    if (r.owned) (void)unpin(r.lo);  // teardown: nowhere to report a failure
  delete ctx;
}

extern "C" int lbf_ctx_num_devices(const lbf_ctx* ctx) {
  if (!ctx) return 0;
  int n = 0;
  for (size_t k = 0; k < ctx->workers.size(); ++k) n += (k == 0 || ctx->workers[k].device != ctx->workers[k - 1].device);
  return n;
}

extern "C" int lbf_ctx_num_workers(const lbf_ctx* ctx) { return ctx ? (int)ctx->workers.size() : 0; }

extern "C" int lbf_ctx_b64_stats(lbf_ctx* ctx, uint64_t* one_pass_chunks, uint64_t* general_chunks) {
  if (!ctx) return fail(LBF_ERR_INVALID, "null context");
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (one_pass_chunks) *one_pass_chunks = ctx->b64_one_pass;
  if (general_chunks) *general_chunks = ctx->b64_general;
  return LBF_OK;
}

extern "C" int lbf_ctx_staging_stats(lbf_ctx* ctx, uint64_t* staged_bytes, uint64_t* direct_bytes) {
  if (!ctx) return fail(LBF_ERR_INVALID, "null context");
  std::lock_guard<std::mutex> lock(ctx->mu);  // between jobs
  uint64_t st = 0, di = 0;
  for (const Worker& w : ctx->workers) st += w.bytes_staged, di += w.bytes_direct;
  if (staged_bytes) *staged_bytes = st;
  if (direct_bytes) *direct_bytes = di;
  return LBF_OK;
}

// Caller-pinned sources: see the pin table above lbf_ctx_create.
extern "C" int lbf_host_register(lbf_ctx* ctx, const void* ptr, uint64_t len) {
  if (!ctx || !ptr || len == 0) return fail(LBF_ERR_INVALID, "lbf_host_register: null context/pointer or empty range");
  const uintptr_t page = (uintptr_t)sysconf(_SC_PAGESIZE);
  const uintptr_t a = reinterpret_cast<uintptr_t>(ptr);
  if (len > UINTPTR_MAX - a - page) return fail(LBF_ERR_INVALID, "lbf_host_register: range wraps");
  Registered r;
  r.user = a;
  r.user_end = a + len;
  r.lo = a & ~(page - 1);
  r.hi = (a + len + page - 1) & ~(page - 1);
  return guarded([&] {
    std::lock_guard<std::mutex> lock(ctx->mu);
    for (const Registered& o : ctx->regs)
      if (r.lo < o.hi && o.lo < r.hi)
        return fail(LBF_ERR_INVALID,
                    "lbf_host_register: range shares pages with one this context already holds (pinning is per "
                    "page: give each registered buffer pages of its own)");
    ctx->regs.reserve(ctx->regs.size() + 1);  // nothing below may throw once pinned
    // Pages a running job pinned on the fly are that job's: it unpins them
    // when it ends.  Taken below for "pinned by someone else", they would
    // leave this registration pointing at pageable memory and its batches
    // copying "directly" from it.  So wait for every such job to
    // end; holding g_autopin_mu from here on keeps a new job from pinning the
    // range before it is in g_pins (reserve_autopin checks that table).
    std::unique_lock<std::mutex> spans(g_autopin_mu);
    g_autopin_cv.wait(spans, [&] { return !autopin_overlaps_locked(r.lo, r.hi); });
    std::lock_guard<std::mutex> pins(g_pin_mu);
    auto next = g_pins.lower_bound(r.lo);
    if (next != g_pins.end() && next->first == r.lo && next->second.hi == r.hi) {
      ++next->second.refs;  // the same range, pinned by another context
      r.owned = true;
      ctx->regs.push_back(r);
      return (int)LBF_OK;
    }
    const bool overlaps = (next != g_pins.end() && next->first < r.hi) ||
                          (next != g_pins.begin() && std::prev(next)->second.hi > r.lo);
    if (overlaps)
      return fail(LBF_ERR_INVALID, "lbf_host_register: range overlaps, but differs from, one another context holds");
    // Pinned already by someone else (a hipHostMalloc'd buffer, a caller's own
    // registration): use it, never unpin it -- but only if ONE pinned
    // allocation covers the caller's whole range.  Its first and last byte
    // being pinned is not enough: they may belong to two neighbouring
    // allocations with pageable memory between them, which a direct copy would
    // then read.  The caller's bytes [a, a + len) are what is checked (a
    // buffer pinned whole by the caller need not end on a page boundary).
    const uint64_t uend = a + len;
    const PinnedAlloc first = pinned_alloc(a), last = pinned_alloc(uend - 1);
    if ((first.pinned && first.end && first.base <= a && uend <= first.end) ||
        (first.pinned && last.pinned && first.id && first.id == last.id)) {
      ctx->regs.push_back(r);
      return (int)LBF_OK;
    }
    if (first.pinned && !first.end && !first.id)
      return fail(LBF_ERR_INVALID,
                  "lbf_host_register: range is pinned already, but HIP does not report the extent of the pinned "
                  "allocation holding it, so it cannot be shown to cover the range");
    if (first.pinned || last.pinned)
      return fail(LBF_ERR_INVALID,
                  "lbf_host_register: range is partly pinned already (no single pinned allocation holds all of it)");
    KeepCurrentDevice keep;
    LBF_HIP_TRY(hipSetDevice(ctx->workers[0].device));
    const hipError_t e = hipHostRegister(reinterpret_cast<void*>(r.lo), r.hi - r.lo, hipHostRegisterPortable);
    if (e == hipErrorHostMemoryAlreadyRegistered) {
      // pages inside the range are pinned by another allocation while its
      // first and last are not (checked above): partly pinned
      (void)hipGetLastError();
      return fail(LBF_ERR_INVALID, "lbf_host_register: range is partly pinned already (pages inside it belong to "
                                   "another pinned allocation)");
    } else if (e != hipSuccess) {
      return hip_fail(e, "hipHostRegister");
    } else {
      g_pins[r.lo] = Pin{r.hi, 1};
      r.owned = true;
    }
    ctx->regs.push_back(r);
    return (int)LBF_OK;
  });
}

extern "C" int lbf_host_unregister(lbf_ctx* ctx, const void* ptr) {
  if (!ctx || !ptr) return fail(LBF_ERR_INVALID, "lbf_host_unregister: null context/pointer");
  std::lock_guard<std::mutex> lock(ctx->mu);  // no job is reading it
  const uintptr_t a = reinterpret_cast<uintptr_t>(ptr);
  for (size_t k = 0; k < ctx->regs.size(); ++k) {
    if (ctx->regs[k].user != a) continue;
    const Registered r = ctx->regs[k];
    ctx->regs.erase(ctx->regs.begin() + (long)k);
    return r.owned ? unpin(r.lo) : LBF_OK;
  }
  return fail(LBF_ERR_INVALID, "lbf_host_unregister: pointer was not registered with this context");
}

extern "C" int lbf_sha1_batch(lbf_ctx* ctx, const uint8_t* base, uint64_t base_len, const uint64_t* offsets,
                              const uint32_t* sizes, uint64_t n, uint8_t* out_digests, int flags) {
  if (!ctx) return fail(LBF_ERR_INVALID, "null context");
  if (n == 0) return LBF_OK;
  if (!base || !offsets || !sizes || !out_digests) return fail(LBF_ERR_INVALID, "null argument");
  if (flags == LBF_DEVICE_PTR) return run_device_job(ctx, base, offsets, sizes, n, out_digests, nullptr, nullptr);
  if (flags != LBF_HOST_PTR) return fail(LBF_ERR_INVALID, "unknown flags");
  Job job{};
  job.src.base = base;
  job.src.base_len = base_len;
  job.offsets = offsets;
  job.sizes = sizes;
  job.digests = out_digests;
  if (int rc = validate_memory_job(job, n)) return rc;
  return guarded([&] { return run_job(ctx, job, n); });
}

extern "C" int lbf_verify_batch(lbf_ctx* ctx, const uint8_t* base, uint64_t base_len, const uint64_t* offsets,
                                const uint32_t* sizes, uint64_t n, const uint8_t* expected, uint8_t* verdicts,
                                int flags) {
  if (!ctx) return fail(LBF_ERR_INVALID, "null context");
  if (n == 0) return LBF_OK;
  if (!base || !offsets || !sizes || !expected || !verdicts) return fail(LBF_ERR_INVALID, "null argument");
  if (flags == LBF_DEVICE_PTR) return run_device_job(ctx, base, offsets, sizes, n, nullptr, expected, verdicts);
  if (flags != LBF_HOST_PTR) return fail(LBF_ERR_INVALID, "unknown flags");
  Job job{};
  job.src.base = base;
  job.src.base_len = base_len;
  job.offsets = offsets;
  job.sizes = sizes;
  job.expected = expected;
  job.verdicts = verdicts;
  if (int rc = validate_memory_job(job, n)) return rc;
  return guarded([&] { return run_job(ctx, job, n); });
}

namespace {

// Files one job holds open at once: a quarter of the soft RLIMIT_NOFILE, so a
// caller with sockets and other descriptors still has room (EncodeFile opens
// one file at a time in the reference, Encoder.cpp:40-79); LBF_FILES_WINDOW
// overrides.  A flood with more files runs as one job per window of files.
uint32_t files_window() {
  if (uint64_t w = env_u64("LBF_FILES_WINDOW", 0)) return (uint32_t)std::min<uint64_t>(w, 1u << 20);
  rlimit rl{};
  uint64_t soft = 1024;
  if (getrlimit(RLIMIT_NOFILE, &rl) == 0 && rl.rlim_cur != RLIM_INFINITY) soft = rl.rlim_cur;
  return (uint32_t)std::max<uint64_t>(4, std::min<uint64_t>(4096, soft / 4));
}

// One job over files [0, n_files) of `paths`, all opened up front.
int files_ranges_job(lbf_ctx* ctx, const char* const* paths, uint32_t n_files, const uint32_t* file_of,
                     const uint64_t* offsets, const uint32_t* sizes, uint64_t n, const uint8_t* expected,
                     uint8_t* out) {
  Job job{};
  job.src.fds.assign(n_files, -1);
  struct Closer {  // every opened file is closed on every path
    std::vector<int>& fds;
    ~Closer() {
      for (int fd : fds)
        if (fd >= 0) close(fd);
    }
  } closer{job.src.fds};
  for (uint32_t f = 0; f < n_files; ++f) {
    const int fd = open(paths[f], O_RDONLY | O_CLOEXEC);
    if (fd < 0) {
      // Out of descriptors is this process's state, not the file's: an error
      // in both modes, never verdict 0 (which would queue the chunks for
      // re-download and overwrite).
      if (errno == EMFILE || errno == ENFILE)
        return fail(LBF_ERR_IO, std::string("cannot open ") + paths[f] + ": too many open files");
      // hash mode needs every file; verify mode leaves a missing file's chunks
      // '0' (Flood.cpp:257)
      if (!expected) return fail(LBF_ERR_IO, std::string("cannot open ") + paths[f]);
    }
    if (fd >= 0) posix_fadvise(fd, 0, 0, POSIX_FADV_SEQUENTIAL);
    job.src.fds[f] = fd;
  }
  if (std::all_of(job.src.fds.begin(), job.src.fds.end(), [](int fd) { return fd < 0; })) {
    memset(out, 0, n);  // verify mode, no file there: every chunk stays '0'
    return LBF_OK;
  }
  job.file_of = file_of;
  job.offsets = offsets;
  job.sizes = sizes;
  job.expected = expected;
  if (expected) job.verdicts = out;
  else job.digests = out;
  return run_job(ctx, job, n);
}

}  // namespace

extern "C" int lbf_files_ranges(lbf_ctx* ctx, const char* const* paths, uint32_t n_files, const uint32_t* file_of,
                                const uint64_t* offsets, const uint32_t* sizes, uint64_t n, const uint8_t* expected,
                                uint8_t* out) {
  if (!ctx || !paths || n_files == 0) return fail(LBF_ERR_INVALID, "null context/paths or no file");
  if (n == 0) return LBF_OK;
  if (!offsets || !sizes || !out || (n_files > 1 && !file_of)) return fail(LBF_ERR_INVALID, "null argument");
  if (file_of)
    for (uint64_t i = 0; i < n; ++i)
      if (file_of[i] >= n_files) return fail(LBF_ERR_INVALID, "chunk " + std::to_string(i) + " names no file");
  for (uint32_t f = 0; f < n_files; ++f)
    if (!paths[f]) return fail(LBF_ERR_INVALID, "null path");
  const uint32_t window = files_window();
  if (n_files <= window || !file_of)
    return guarded([&] { return files_ranges_job(ctx, paths, n_files, file_of, offsets, sizes, n, expected, out); });
  // More files than may be open at once: one job per window of `window`
  // consecutive files, each over that window's chunks (gathered, then the
  // results scattered back to the caller's indices).
  return guarded([&]() -> int {
    const uint32_t n_win = (n_files + window - 1) / window;
    std::vector<std::vector<uint64_t>> members(n_win);
    for (uint64_t i = 0; i < n; ++i) members[file_of[i] / window].push_back(i);
    const size_t per = expected ? 1 : 20;
    std::vector<uint32_t> fo;
    std::vector<uint64_t> offs;
    std::vector<uint32_t> szs;
    std::vector<uint8_t> exp, res;
    for (uint32_t w = 0; w < n_win; ++w) {
      const std::vector<uint64_t>& idx = members[w];
      if (idx.empty()) continue;
      const uint32_t f0 = w * window, nf = std::min(window, n_files - f0);
      fo.resize(idx.size());
      offs.resize(idx.size());
      szs.resize(idx.size());
      res.assign(idx.size() * per, 0);
      if (expected) exp.resize(idx.size() * 20);
      for (size_t k = 0; k < idx.size(); ++k) {
        fo[k] = file_of[idx[k]] - f0;
        offs[k] = offsets[idx[k]];
        szs[k] = sizes[idx[k]];
        if (expected) memcpy(&exp[20 * k], expected + 20 * idx[k], 20);
      }
      if (int rc = files_ranges_job(ctx, paths + f0, nf, fo.data(), offs.data(), szs.data(), idx.size(),
                                    expected ? exp.data() : nullptr, res.data()))
        return rc;
      for (size_t k = 0; k < idx.size(); ++k) memcpy(out + per * idx[k], &res[per * k], per);
    }
    return LBF_OK;
  });
}

extern "C" int lbf_file_ranges(lbf_ctx* ctx, const char* path, const uint64_t* offsets, const uint32_t* sizes,
                               uint64_t n, const uint8_t* expected, uint8_t* out) {
  if (!ctx || !path) return fail(LBF_ERR_INVALID, "null context/path");
  return lbf_files_ranges(ctx, &path, 1, nullptr, offsets, sizes, n, expected, out);
}

namespace {
// The device memory of the two base64 entry points: one allocation on worker
// 0's device (current when this runs), grown on demand; the caller holds ctx->mu.
int b64_scratch(lbf_ctx* ctx, uint64_t need, const char* who) {
  if (need <= ctx->b64_cap) return LBF_OK;
  if (ctx->b64_dev) (void)hipFree(ctx->b64_dev);
  ctx->b64_dev = nullptr;
  ctx->b64_cap = 0;
  const uint64_t want = std::max<uint64_t>(need, 64ull << 20);
  if (hipMalloc(reinterpret_cast<void**>(&ctx->b64_dev), want) != hipSuccess) {
    (void)hipGetLastError();
    return fail(LBF_ERR_NOMEM, std::string(who) + ": device allocation of " + std::to_string(want) + " bytes");
  }
  ctx->b64_cap = want;
  return LBF_OK;
}

// Every exit of a base64 entry point after its first async copy waits for the
// stream, so no copy is still reading a local staging vector or the caller's
// (possibly pinned) buffers, or writing into them, once the call has returned
// (ADVICE r04).  Declared after the host vectors the copies use, so it runs
// before they are destroyed.
struct SyncOnExit {
  hipStream_t st;
  ~SyncOnExit() {
    (void)hipStreamSynchronize(st);
    (void)hipGetLastError();
  }
};

// Caller slots [off[i], off[i] + len[i]) that the device writes back: sorted,
// checked for overlap (two chunks' results in one byte would race on the
// device), and merged into runs of touching slots.  Each run is one D2H; the
// bytes between runs are the caller's and are never written.
struct SlotRun {
  uint64_t lo, hi;
};
int slot_runs(const uint64_t* off, const uint64_t* len, uint64_t n, const char* who, std::vector<SlotRun>& runs) {
  std::vector<uint64_t> idx;
  idx.reserve(n);
  for (uint64_t i = 0; i < n; ++i)
    if (len[i]) idx.push_back(i);
  std::sort(idx.begin(), idx.end(), [&](uint64_t a, uint64_t b) { return off[a] < off[b]; });
  runs.clear();
  for (uint64_t i : idx) {
    if (!runs.empty() && off[i] < runs.back().hi)
      return fail(LBF_ERR_INVALID, std::string(who) + ": slot " + std::to_string(i) + " overlaps another slot");
    if (!runs.empty() && off[i] == runs.back().hi)
      runs.back().hi += len[i];
    else
      runs.push_back(SlotRun{off[i], off[i] + len[i]});
  }
  return LBF_OK;
}
}  // namespace

// The wire kernels keep text and byte positions inside a chunk, and their
// tile counts, in 32 bits (kern_b64.hpp): (len + tile - 1) / tile and
// tile * tile_text must not wrap, so chunks are bounded well below 2^32.  The
// reference's chunks are 64 KiB to a few MiB (Encoder.cpp:17-102); 1 GiB of
// bytes encodes to 1.43 GB of text.  ADVICE r05: past 2^32 the positions
// wrapped and tiles were never launched.
constexpr uint64_t kB64MaxChunk = 1ull << 30, kB64MaxText = 3ull << 29;

extern "C" uint64_t lbf_b64_put_length(uint64_t size) { return 4 * (size / 3) + (size % 3 ? 4 : 0) + size / 3 / 18; }

// Chunks to send: verify on the device (ChunkMethods.cpp:116-123), then encode
// each as the base64 text of its SendChunk frame (XmlRpcValue.cpp:439-452,
// kern_b64.hpp), from the same
// device copy.  Synchronous on worker 0's first stream: one H2D of the bytes'
// span and one of the tables, two launches, one D2H of the verdicts and one of
// the text span.
extern "C" int lbf_verify_encode_b64_batch(lbf_ctx* ctx, const uint8_t* data, uint64_t data_len,
                                           const uint64_t* offsets, const uint32_t* sizes, uint64_t n,
                                           const uint8_t* expected, uint8_t* verdicts, char* text, uint64_t text_len,
                                           const uint64_t* text_offsets) {
  if (!ctx) return fail(LBF_ERR_INVALID, "null context");
  if (n == 0) return LBF_OK;
  if (!data || !offsets || !sizes || !expected || !verdicts || !text || !text_offsets)
    return fail(LBF_ERR_INVALID, "lbf_verify_encode_b64_batch: null argument");
  if (n > 0x7FFFFFFFull) return fail(LBF_ERR_INVALID, "lbf_verify_encode_b64_batch: n too large");
  uint64_t dlo = UINT64_MAX, dhi = 0, tlo = UINT64_MAX, thi = 0;
  for (uint64_t i = 0; i < n; ++i) {
    if (sizes[i] > kB64MaxChunk)
      return fail(LBF_ERR_INVALID, "lbf_verify_encode_b64_batch: chunk " + std::to_string(i) +
                                       " larger than the wire encode takes (1 GiB)");
    if (offsets[i] > data_len || sizes[i] > data_len - offsets[i])
      return fail(LBF_ERR_INVALID, "lbf_verify_encode_b64_batch: chunk " + std::to_string(i) + " outside the buffer");
    const uint64_t tl = lbf_b64_put_length(sizes[i]);
    if (text_offsets[i] > text_len || tl > text_len - text_offsets[i])
      return fail(LBF_ERR_INVALID, "lbf_verify_encode_b64_batch: text slot " + std::to_string(i) + " outside the buffer");
    dlo = std::min(dlo, offsets[i]);
    dhi = std::max(dhi, offsets[i] + sizes[i]);
    tlo = std::min(tlo, text_offsets[i]);
    thi = std::max(thi, text_offsets[i] + tl);
  }
  uint32_t max_size = 0;
  for (uint64_t i = 0; i < n; ++i) max_size = std::max(max_size, sizes[i]);
  std::vector<uint64_t> tlens(n);
  for (uint64_t i = 0; i < n; ++i) tlens[i] = lbf_b64_put_length(sizes[i]);
  std::vector<SlotRun> runs;  // the text slots the D2H writes, and nothing between them
  if (int rc = slot_runs(text_offsets, tlens.data(), n, "lbf_verify_encode_b64_batch", runs)) return rc;
  dlo &= ~15ull;  // device offsets keep the host offsets' alignment mod 16
  tlo &= ~15ull;
  return guarded([&] {
    auto up = [](uint64_t x, uint64_t a) { return (x + a - 1) / a * a; };
    std::vector<uint8_t> in(n * (8 + 8 + 4 + 20));
    uint64_t* doff = reinterpret_cast<uint64_t*>(in.data());
    uint64_t* toff = doff + n;
    uint32_t* sz = reinterpret_cast<uint32_t*>(toff + n);
    for (uint64_t i = 0; i < n; ++i) {
      doff[i] = offsets[i] - dlo;
      toff[i] = text_offsets[i] - tlo;
      sz[i] = sizes[i];
    }
    memcpy(sz + n, expected, 20 * n);
    // device layout: bytes | text | inputs (offsets, text offsets, sizes, expected) | verdicts
    const uint64_t data_b = up(dhi - dlo + 16, 256), text_b = up(thi - tlo + 16, 256), in_b = up(in.size(), 256);
    const uint64_t need = data_b + text_b + in_b + up(n, 256);
    std::lock_guard<std::mutex> lock(ctx->mu);
    KeepCurrentDevice keep;
    Worker& w = ctx->workers[0];
    LBF_HIP_TRY(hipSetDevice(w.device));
    if (int rc = b64_scratch(ctx, need, "lbf_verify_encode_b64_batch")) return rc;
    uint8_t* d_data = ctx->b64_dev;
    uint8_t* d_text = d_data + data_b;
    uint8_t* d_in = d_text + text_b;
    uint8_t* d_ver = d_in + in_b;
    hipStream_t st = w.dev[0].stream;
    SyncOnExit sync{st};
    if (dhi > dlo) LBF_HIP_TRY(hipMemcpyAsync(d_data, data + dlo, dhi - dlo, hipMemcpyHostToDevice, st));
    LBF_HIP_TRY(hipMemcpyAsync(d_in, in.data(), in.size(), hipMemcpyHostToDevice, st));
    const uint64_t* d_doff = reinterpret_cast<const uint64_t*>(d_in);
    const uint64_t* d_toff = d_doff + n;
    const uint32_t* d_sz = reinterpret_cast<const uint32_t*>(d_toff + n);
    const uint8_t* d_exp = reinterpret_cast<const uint8_t*>(d_sz + n);
    if (int rc = lbf_sha1_launch(d_data, d_doff, d_sz, n, nullptr, d_exp, d_ver, st)) return rc;
    if (int rc = lbf::launch_b64_encode(d_data, d_doff, d_sz, d_text, d_toff, (uint32_t)n, max_size, st)) return rc;
    LBF_HIP_TRY(hipMemcpyAsync(verdicts, d_ver, n, hipMemcpyDeviceToHost, st));
    for (const SlotRun& r : runs)
      LBF_HIP_TRY(hipMemcpyAsync(text + r.lo, d_text + (r.lo - tlo), r.hi - r.lo, hipMemcpyDeviceToHost, st));
    LBF_HIP_TRY(hipStreamSynchronize(st));
    return (int)LBF_OK;
  });
}

// Received chunks as base64 text: decode on the device (kern_b64.hpp), then
// the shipped hash kernels verify the decoded bytes in HBM.  Synchronous on
// worker 0's first stream: one H2D of the text span and one of the tables, two
// launches, one D2H of the results and one of the decoded span.
extern "C" int lbf_b64_verify_batch(lbf_ctx* ctx, const char* text, uint64_t text_len,
                                    const uint64_t* text_offsets, const uint32_t* text_lens, uint64_t n,
                                    const uint32_t* expected_sizes, const uint8_t* expected, uint8_t* out,
                                    uint64_t out_len, const uint64_t* out_offsets, uint32_t* out_sizes,
                                    uint8_t* verdicts) {
  if (!ctx) return fail(LBF_ERR_INVALID, "null context");
  if (n == 0) return LBF_OK;
  if (!text || !text_offsets || !text_lens || !expected_sizes || !expected || !verdicts)
    return fail(LBF_ERR_INVALID, "lbf_b64_verify_batch: null argument");
  if (out && !out_offsets) return fail(LBF_ERR_INVALID, "lbf_b64_verify_batch: out without out_offsets");
  if (n > 0x7FFFFFFFull) return fail(LBF_ERR_INVALID, "lbf_b64_verify_batch: n too large");
  uint64_t tlo = UINT64_MAX, thi = 0, olo = UINT64_MAX, ohi = 0;
  for (uint64_t i = 0; i < n; ++i) {
    if (text_lens[i] > kB64MaxText || expected_sizes[i] > kB64MaxChunk)
      return fail(LBF_ERR_INVALID, "lbf_b64_verify_batch: chunk " + std::to_string(i) +
                                       " larger than the wire decode takes (1 GiB of bytes, 1.5 GiB of text)");
    if (text_offsets[i] > text_len || text_lens[i] > text_len - text_offsets[i])
      return fail(LBF_ERR_INVALID, "lbf_b64_verify_batch: text range " + std::to_string(i) + " outside the buffer");
    tlo = std::min(tlo, text_offsets[i]);
    thi = std::max(thi, text_offsets[i] + text_lens[i]);
    if (out) {
      if (out_offsets[i] > out_len || expected_sizes[i] > out_len - out_offsets[i])
        return fail(LBF_ERR_INVALID, "lbf_b64_verify_batch: output slot " + std::to_string(i) + " outside the buffer");
      olo = std::min(olo, out_offsets[i]);
      ohi = std::max(ohi, out_offsets[i] + expected_sizes[i]);
    }
  }
  // device offsets keep the host offsets' alignment mod 16; the D2H writes the
  // output slots and nothing between them
  std::vector<SlotRun> runs;
  if (out) {
    std::vector<uint64_t> olens(expected_sizes, expected_sizes + n);
    if (int rc = slot_runs(out_offsets, olens.data(), n, "lbf_b64_verify_batch", runs)) return rc;
  }
  uint32_t max_tlen = 0, max_cap = 0;
  for (uint64_t i = 0; i < n; ++i) {
    max_tlen = std::max(max_tlen, text_lens[i]);
    max_cap = std::max(max_cap, expected_sizes[i]);
  }
  tlo &= ~15ull;
  if (out) olo &= ~15ull;
  return guarded([&] {
    auto up = [](uint64_t x, uint64_t a) { return (x + a - 1) / a * a; };
    std::vector<uint64_t> toff(n), soff(n), ooff(n);
    std::vector<uint32_t> tlen(n), cap(n);
    uint64_t sext = 0, outb = 0;
    for (uint64_t i = 0; i < n; ++i) {
      toff[i] = text_offsets[i] - tlo;
      soff[i] = sext;
      sext += up(text_lens[i], 16);
      tlen[i] = text_lens[i];
      cap[i] = expected_sizes[i];
      if (out) {
        ooff[i] = out_offsets[i] - olo;
      } else {
        ooff[i] = outb;
        outb += up(expected_sizes[i], 16);
      }
    }
    if (out) outb = ohi - olo;
    // device layout: text | sextets | bytes | inputs (offsets, lengths, caps, expected) then, right behind
    // them, the results (sizes, over, verdicts, redo flags): one H2D carries the inputs and the zeroed
    // results, one D2H brings the results back
    const uint64_t kIn = 8 * 3 + 4 * 2 + 20, kRes = 4 + 1 + 1 + 1;  // bytes per chunk; kIn * n keeps 4-byte alignment
    const uint64_t text_b = up(thi - tlo, 256), sext_b = up(sext, 256), out_b = up(outb + 16, 256);
    const uint64_t io_b = up(n * (kIn + kRes), 256);
    const uint64_t need = text_b + sext_b + out_b + io_b;
    std::lock_guard<std::mutex> lock(ctx->mu);
    KeepCurrentDevice keep;
    Worker& w = ctx->workers[0];
    LBF_HIP_TRY(hipSetDevice(w.device));
    if (int rc = b64_scratch(ctx, need, "lbf_b64_verify_batch")) return rc;
    uint8_t* d_text = ctx->b64_dev;
    uint8_t* d_sext = d_text + text_b;
    uint8_t* d_out = d_sext + sext_b;
    uint8_t* d_in = d_out + out_b;
    uint8_t* d_res = d_in + kIn * n;
    std::vector<uint8_t> in(n * (kIn + kRes), 0);
    uint8_t* q = in.data();
    auto put = [&](const void* src, uint64_t bytes) {
      memcpy(q, src, bytes);
      q += bytes;
    };
    put(toff.data(), 8 * n);
    put(soff.data(), 8 * n);
    put(ooff.data(), 8 * n);
    put(tlen.data(), 4 * n);
    put(cap.data(), 4 * n);
    put(expected, 20 * n);
    hipStream_t st = w.dev[0].stream;
    std::vector<uint8_t> res(n * kRes);
    SyncOnExit sync{st};
    if (thi > tlo) LBF_HIP_TRY(hipMemcpyAsync(d_text, text + tlo, thi - tlo, hipMemcpyHostToDevice, st));
    LBF_HIP_TRY(hipMemcpyAsync(d_in, in.data(), in.size(), hipMemcpyHostToDevice, st));
    const uint64_t* d_toff = reinterpret_cast<const uint64_t*>(d_in);
    const uint64_t* d_soff = d_toff + n;
    const uint64_t* d_ooff = d_soff + n;
    const uint32_t* d_tlen = reinterpret_cast<const uint32_t*>(d_ooff + n);
    const uint32_t* d_cap = d_tlen + n;
    const uint8_t* d_exp = reinterpret_cast<const uint8_t*>(d_cap + n);
    uint32_t* d_sizes = reinterpret_cast<uint32_t*>(d_res);
    uint8_t* d_over = reinterpret_cast<uint8_t*>(d_sizes + n);
    uint8_t* d_ver = d_over + n;
    uint8_t* d_redo = d_ver + n;  // uploaded as zeros
    lbf::B64Launch b{d_text, d_sext, d_toff, d_soff, d_tlen, d_out,   d_ooff, d_cap,
                     d_sizes, d_over, d_redo, (uint32_t)n, max_tlen, max_cap};
    if (int rc = lbf::launch_b64_decode(b, st)) return rc;
    // the decoded lengths are the chunk sizes the hash kernels read
    if (int rc = lbf_sha1_launch(d_out, d_ooff, d_sizes, n, nullptr, d_exp, d_ver, st)) return rc;
    LBF_HIP_TRY(hipMemcpyAsync(res.data(), d_res, res.size(), hipMemcpyDeviceToHost, st));
    for (const SlotRun& r : runs)
      LBF_HIP_TRY(hipMemcpyAsync(out + r.lo, d_out + (r.lo - olo), r.hi - r.lo, hipMemcpyDeviceToHost, st));
    LBF_HIP_TRY(hipStreamSynchronize(st));
    const uint8_t* redo = res.data() + 6 * n;
    uint64_t general = 0;
    for (uint64_t i = 0; i < n; ++i) general += redo[i] != 0;
    ctx->b64_general += general;
    ctx->b64_one_pass += n - general;
    const uint32_t* sizes = reinterpret_cast<const uint32_t*>(res.data());
    const uint8_t* over = res.data() + 4 * n;
    const uint8_t* ver = over + n;
    for (uint64_t i = 0; i < n; ++i) {
      // ChunkMethods.cpp:156: the decoded length must be the chunk's size
      const bool longer = over[i] != 0;
      verdicts[i] = (ver[i] && !longer && sizes[i] == expected_sizes[i]) ? 1 : 0;
      if (out_sizes) out_sizes[i] = longer ? expected_sizes[i] + 1 : sizes[i];
    }
    return (int)LBF_OK;
  });
}

extern "C" int lbf_sha1_one(lbf_ctx* ctx, const uint8_t* data, uint32_t size, uint8_t out[20]) {
  static const uint8_t kEmpty = 0;
  if (!data && size) return fail(LBF_ERR_INVALID, "null data");
  const uint64_t off = 0;
  return lbf_sha1_batch(ctx, data ? data : &kEmpty, size, &off, &size, 1, out, LBF_HOST_PTR);
}
