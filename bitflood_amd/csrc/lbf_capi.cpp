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
#include <fcntl.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <string>
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
  return fail(e == hipErrorOutOfMemory ? LBF_ERR_NOMEM : LBF_ERR_HIP,
              std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace lbf

using lbf::fail;

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
// Context: per-device workers with LBF_SLOTS pipeline slots each.
// ---------------------------------------------------------------------------
namespace {

struct Slot {
  hipStream_t stream = nullptr;
  uint8_t* d_data = nullptr;       // slot_bytes
  uint64_t* d_off = nullptr;       // desc_cap
  uint32_t* d_size = nullptr;
  uint8_t* d_dig = nullptr;        // desc_cap * 20
  uint8_t* d_exp = nullptr;
  uint8_t* d_ver = nullptr;        // desc_cap
  uint8_t* h_data = nullptr;       // pinned, slot_bytes
  uint64_t* h_off = nullptr;       // pinned
  uint32_t* h_size = nullptr;
  uint8_t* h_dig = nullptr;
  uint8_t* h_exp = nullptr;
  uint8_t* h_ver = nullptr;
  uint8_t* h_ok = nullptr;         // 1 = chunk bytes fully available
  // pending group to finalize after the stream drains
  bool pending = false;
  uint64_t g_begin = 0, g_end = 0;
};

struct Worker {
  int device = 0;
  std::vector<Slot> slot;  // LBF_SLOTS of them (default 3), used round-robin
  uint64_t slot_bytes = 0;  // current staging capacity per slot (grown on demand)
  uint64_t slot_max = 0;    // LBF_SLOT_MB: the largest a slot may grow
  uint64_t desc_cap = 0;
};

}  // namespace

struct lbf_ctx {
  std::vector<Worker> workers;
  std::mutex mu;
};

namespace {

uint64_t env_u64(const char* name, uint64_t dflt) {
  const char* v = getenv(name);
  if (!v || !*v) return dflt;
  return strtoull(v, nullptr, 10);
}

// Staging memory is sized to the work, not reserved up front: pinning 2 x 512
// MiB costs ≈200 ms at context creation and ≈110 ms at destruction
// (tools/startup_probe.py), which a one-chunk Base64Encode or a small file
// should not pay.  A slot grows, never shrinks, in 8 MiB steps up to slot_max.
constexpr uint64_t kSlotStep = 8ull << 20;

int ensure_slot_bytes(Worker& w, uint64_t need) {
  need = std::min(w.slot_max, (std::max(need, kSlotStep) + kSlotStep - 1) / kSlotStep * kSlotStep);
  if (need <= w.slot_bytes) return LBF_OK;
  for (Slot& s : w.slot) {
    LBF_HIP_TRY(hipStreamSynchronize(s.stream));
    if (s.d_data) (void)hipFree(s.d_data);
    if (s.h_data) (void)hipHostFree(s.h_data);
    s.d_data = nullptr;
    s.h_data = nullptr;
  }
  w.slot_bytes = 0;
  for (Slot& s : w.slot) {
    LBF_HIP_TRY(hipMalloc((void**)&s.d_data, need));
    LBF_HIP_TRY(hipHostMalloc((void**)&s.h_data, need, hipHostMallocDefault));
  }
  w.slot_bytes = need;
  return LBF_OK;
}

int worker_init(Worker& w, int device) {
  w.device = device;
  w.slot_max = std::max<uint64_t>(env_u64("LBF_SLOT_MB", 512) << 20, 1ull << 20);
  // Three slots keep the PCIe link busy: with two, staging group g+2 waits for
  // group g's H2D *and* its kernel (one chunk's serial chain, ≈3.2 ms at 256 KiB
  // whatever the group size), so the link idles once per pair of groups.
  w.slot.resize(std::min<uint64_t>(8, std::max<uint64_t>(2, env_u64("LBF_SLOTS", 3))));
  w.slot_bytes = 0;
  w.desc_cap = 1u << 16;
  LBF_HIP_TRY(hipSetDevice(device));
  for (Slot& s : w.slot) {
    LBF_HIP_TRY(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
    LBF_HIP_TRY(hipMalloc((void**)&s.d_off, w.desc_cap * 8));
    LBF_HIP_TRY(hipMalloc((void**)&s.d_size, w.desc_cap * 4));
    LBF_HIP_TRY(hipMalloc((void**)&s.d_dig, w.desc_cap * 20));
    LBF_HIP_TRY(hipMalloc((void**)&s.d_exp, w.desc_cap * 20));
    LBF_HIP_TRY(hipMalloc((void**)&s.d_ver, w.desc_cap));
    LBF_HIP_TRY(hipHostMalloc((void**)&s.h_off, w.desc_cap * 8, hipHostMallocDefault));
    LBF_HIP_TRY(hipHostMalloc((void**)&s.h_size, w.desc_cap * 4, hipHostMallocDefault));
    LBF_HIP_TRY(hipHostMalloc((void**)&s.h_dig, w.desc_cap * 20, hipHostMallocDefault));
    LBF_HIP_TRY(hipHostMalloc((void**)&s.h_exp, w.desc_cap * 20, hipHostMallocDefault));
    LBF_HIP_TRY(hipHostMalloc((void**)&s.h_ver, w.desc_cap, hipHostMallocDefault));
    s.h_ok = new uint8_t[w.desc_cap];
  }
  return LBF_OK;
}

void worker_free(Worker& w) {
  if (hipSetDevice(w.device) != hipSuccess) return;
  for (Slot& s : w.slot) {
    // teardown: errors here have nowhere to go, the context is being destroyed
    if (s.stream) (void)hipStreamSynchronize(s.stream);
    for (void* d : {(void*)s.d_data, (void*)s.d_off, (void*)s.d_size, (void*)s.d_dig, (void*)s.d_exp, (void*)s.d_ver})
      (void)hipFree(d);
    for (void* h : {(void*)s.h_data, (void*)s.h_off, (void*)s.h_size, (void*)s.h_dig, (void*)s.h_exp, (void*)s.h_ver})
      (void)hipHostFree(h);
    delete[] s.h_ok;
    if (s.stream) (void)hipStreamDestroy(s.stream);
    s = Slot{};
  }
}

// Host threads per staging copy: LBF_COPY_THREADS, default 8 (a GPU box's
// share of host cores is 16; two devices' workers may copy at once).
unsigned copy_threads() {
  static const unsigned n = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(64, env_u64("LBF_COPY_THREADS", 8)));
  return n;
}

// Where a job's bytes come from: caller memory (bounds-checked up front) or a
// file read with pread.  read() returns the bytes actually available.
struct Source {
  const uint8_t* base = nullptr;  // memory source
  uint64_t base_len = 0;
  int fd = -1;                    // file source
  unsigned threads = copy_threads();  // staging copy threads

  uint64_t read_serial(uint8_t* dst, uint64_t off, uint64_t len) const {
    if (fd < 0) {
      memcpy(dst, base + off, len);
      return len;
    }
    uint64_t got = 0;
    while (got < len) {
      const ssize_t r = pread(fd, dst + got, len - got, (off_t)(off + got));
      if (r <= 0) break;  // EOF or error: the rest is unavailable
      got += (uint64_t)r;
    }
    return got;
  }

  // A single host thread copies ~17 GiB/s into pinned memory, a third of what
  // PCIe Gen5 moves, so large ranges are split over `threads` contiguous
  // parts.  Returns the length of the readable prefix, as read_serial does.
  uint64_t read(uint8_t* dst, uint64_t off, uint64_t len) const {
    constexpr uint64_t kMinPart = 8ull << 20;
    const uint64_t parts = std::min<uint64_t>(threads, len / kMinPart);
    if (parts <= 1) return read_serial(dst, off, len);
    // ceil(len / parts), rounded up to a page: parts * step must cover len.
    // (Rounding floor(len / parts) instead left the last len % parts bytes
    // uncopied whenever floor(len / parts) was already a page multiple; found
    // by tools/fuzz_gpu.py, regression test test_staging_split_covers_tail.)
    const uint64_t step = ((len + parts - 1) / parts + 4095) & ~4095ull;
    std::vector<uint64_t> got(parts, 0), want(parts, 0);
    std::vector<std::thread> th;
    for (uint64_t p = 0; p < parts; ++p) {
      const uint64_t a = p * step;
      if (a >= len) break;
      want[p] = std::min(step, len - a);
      th.emplace_back([&, p, a] { got[p] = read_serial(dst + a, off + a, want[p]); });
    }
    for (auto& t : th) t.join();
    uint64_t total = 0;
    for (uint64_t p = 0; p < parts; ++p) {
      total += got[p];
      if (got[p] < want[p]) break;
    }
    return total;
  }
};

struct Job {
  Source src;
  const uint64_t* offsets;
  const uint32_t* sizes;
  const uint8_t* expected;  // null => hash mode
  uint8_t* digests;         // hash mode output
  uint8_t* verdicts;        // verify mode output
};

// Copy finished results of a slot's group to the caller's arrays.  Chunks that
// were not fully readable: verdict 0 (verify) or an LBF_ERR_IO (hash).
int finalize(const Job& job, Slot& s) {
  if (!s.pending) return LBF_OK;
  s.pending = false;
  const uint64_t cnt = s.g_end - s.g_begin;
  if (job.expected) {
    for (uint64_t k = 0; k < cnt; ++k) job.verdicts[s.g_begin + k] = s.h_ver[k] & s.h_ok[k];
    return LBF_OK;
  }
  for (uint64_t k = 0; k < cnt; ++k)
    if (!s.h_ok[k]) return fail(LBF_ERR_IO, "chunk " + std::to_string(s.g_begin + k) + " could not be read in full");
  memcpy(job.digests + 20 * s.g_begin, s.h_dig, cnt * 20);
  return LBF_OK;
}

// One chunk that does not fit a slot: a dedicated device buffer.
int run_oversize(Worker& w, const Job& job, uint64_t i) {
  Slot& s = w.slot[0];
  LBF_HIP_TRY(hipStreamSynchronize(s.stream));
  const uint32_t sz = job.sizes[i];
  std::vector<uint8_t> host(sz ? sz : 1);
  const bool ok = job.src.read(host.data(), job.offsets[i], sz) == sz;
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
    s.h_off[0] = 0;
    s.h_size[0] = sz;
    if (hipMemcpy(d, host.data(), sz, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(s.d_off, s.h_off, 8, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(s.d_size, s.h_size, 4, hipMemcpyHostToDevice) != hipSuccess) {
      rc = fail(LBF_ERR_HIP, "oversize chunk H2D failed");
      break;
    }
    if (job.expected && hipMemcpy(s.d_exp, job.expected + 20 * i, 20, hipMemcpyHostToDevice) != hipSuccess) {
      rc = fail(LBF_ERR_HIP, "oversize expected H2D failed");
      break;
    }
    rc = lbf_sha1_launch(d, s.d_off, s.d_size, 1, job.expected ? nullptr : s.d_dig,
                         job.expected ? s.d_exp : nullptr, job.expected ? s.d_ver : nullptr, s.stream);
    if (rc) break;
    if (hipStreamSynchronize(s.stream) != hipSuccess) {
      rc = fail(LBF_ERR_HIP, "oversize kernel failed");
      break;
    }
    const hipError_t e = job.expected ? hipMemcpy(job.verdicts + i, s.d_ver, 1, hipMemcpyDeviceToHost)
                                      : hipMemcpy(job.digests + 20 * i, s.d_dig, 20, hipMemcpyDeviceToHost);
    if (e != hipSuccess) rc = fail(LBF_ERR_HIP, "oversize D2H failed");
  } while (0);
  (void)hipFree(d);
  return rc;
}

// Process descriptors [begin, end) on one device.  Groups of consecutive
// descriptors whose covering byte range fits a slot are staged into pinned
// memory (memcpy or pread), then H2D + kernel + D2H run on the slot's stream
// while the host stages the next group into the other slot.
int worker_run(Worker& w, const Job& job, uint64_t begin, uint64_t end) {
  LBF_HIP_TRY(hipSetDevice(w.device));
  {
    // Staging sized to the byte range this worker covers: a quarter of it per
    // slot once it exceeds kSplitMin, so a mid-sized job still runs as several
    // groups whose copies, H2Ds and kernels overlap; never below the largest
    // chunk that fits a slot, and capped at slot_max.
    constexpr uint64_t kSplitMin = 32ull << 20;
    uint64_t lo = UINT64_MAX, hi = 0, largest = 0;
    for (uint64_t k = begin; k < end; ++k)
      if ((uint64_t)job.sizes[k] + 15 <= w.slot_max) {
        lo = std::min(lo, job.offsets[k]);
        hi = std::max(hi, job.offsets[k] + job.sizes[k]);
        largest = std::max<uint64_t>(largest, job.sizes[k]);
      }
    const uint64_t span = hi > lo ? hi - lo : 0;
    const uint64_t per = span <= kSplitMin ? span : std::max({kSplitMin, (span + 3) / 4, largest});
    if (end > begin)
      if (int rc = ensure_slot_bytes(w, std::min(per, w.slot_max) + 16)) return rc;
  }
  int cur = 0;
  uint64_t i = begin;
  int rc = LBF_OK;
  while (i < end && rc == LBF_OK) {
    if ((uint64_t)job.sizes[i] + 15 > w.slot_bytes) {
      for (Slot& s : w.slot) {
        LBF_HIP_TRY(hipStreamSynchronize(s.stream));
        if ((rc = finalize(job, s))) break;
      }
      if (rc == LBF_OK) rc = run_oversize(w, job, i);
      ++i;
      continue;
    }
    uint64_t lo = job.offsets[i], hi = lo + job.sizes[i];
    uint64_t j = i + 1;
    while (j < end && j - i < w.desc_cap) {
      const uint64_t o = job.offsets[j], e = o + job.sizes[j];
      const uint64_t nlo = std::min(lo, o), nhi = std::max(hi, e);
      if (nhi - nlo + 15 > w.slot_bytes) break;
      lo = nlo;
      hi = nhi;
      ++j;
    }
    Slot& s = w.slot[cur];
    LBF_HIP_TRY(hipStreamSynchronize(s.stream));
    if ((rc = finalize(job, s))) break;
    const uint64_t cnt = j - i;
    // The covered range [lo, hi) lands at h_data + (lo % 16) so each chunk
    // keeps its offset's 16-byte phase (aligned chunks take the vector-load
    // path on the device).
    const uint64_t shift = lo & 15u;
    const uint64_t avail = job.src.read(s.h_data + shift, lo, hi - lo);
    for (uint64_t k = 0; k < cnt; ++k) {
      const uint64_t o = job.offsets[i + k];
      s.h_off[k] = o - lo + shift;
      s.h_size[k] = job.sizes[i + k];
      // An empty chunk is always readable, wherever it lies: the reference's
      // fseek succeeds past EOF and fread of 0 bytes returns 0 (Flood.cpp:259-275).
      s.h_ok[k] = (job.sizes[i + k] == 0 || o + job.sizes[i + k] <= lo + avail) ? 1 : 0;
    }
    const uint64_t copy_bytes = avail + shift;
    LBF_HIP_TRY(hipMemcpyAsync(s.d_data, s.h_data, copy_bytes, hipMemcpyHostToDevice, s.stream));
    LBF_HIP_TRY(hipMemcpyAsync(s.d_off, s.h_off, cnt * 8, hipMemcpyHostToDevice, s.stream));
    LBF_HIP_TRY(hipMemcpyAsync(s.d_size, s.h_size, cnt * 4, hipMemcpyHostToDevice, s.stream));
    // Unreadable chunks must not be hashed from stale slot bytes past `avail`:
    // give them size 0 on the device (their result is discarded anyway).
    bool any_short = false;
    for (uint64_t k = 0; k < cnt; ++k) any_short |= !s.h_ok[k];
    if (any_short) {
      for (uint64_t k = 0; k < cnt; ++k)
        if (!s.h_ok[k]) {
          s.h_size[k] = 0;
          s.h_off[k] = 0;
        }
      LBF_HIP_TRY(hipMemcpyAsync(s.d_off, s.h_off, cnt * 8, hipMemcpyHostToDevice, s.stream));
      LBF_HIP_TRY(hipMemcpyAsync(s.d_size, s.h_size, cnt * 4, hipMemcpyHostToDevice, s.stream));
    }
    if (job.expected) {
      memcpy(s.h_exp, job.expected + 20 * i, cnt * 20);
      LBF_HIP_TRY(hipMemcpyAsync(s.d_exp, s.h_exp, cnt * 20, hipMemcpyHostToDevice, s.stream));
      rc = lbf_sha1_launch(s.d_data, s.d_off, s.d_size, cnt, nullptr, s.d_exp, s.d_ver, s.stream);
      if (rc) break;
      LBF_HIP_TRY(hipMemcpyAsync(s.h_ver, s.d_ver, cnt, hipMemcpyDeviceToHost, s.stream));
    } else {
      rc = lbf_sha1_launch(s.d_data, s.d_off, s.d_size, cnt, s.d_dig, nullptr, nullptr, s.stream);
      if (rc) break;
      LBF_HIP_TRY(hipMemcpyAsync(s.h_dig, s.d_dig, cnt * 20, hipMemcpyDeviceToHost, s.stream));
    }
    s.pending = true;
    s.g_begin = i;
    s.g_end = j;
    cur = (cur + 1) % (int)w.slot.size();
    i = j;
  }
  for (Slot& s : w.slot) {
    if (hipStreamSynchronize(s.stream) != hipSuccess && rc == LBF_OK)
      rc = fail(LBF_ERR_HIP, "stream synchronize failed");
    if (rc == LBF_OK) rc = finalize(job, s);
    s.pending = false;
  }
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

int run_job(lbf_ctx* ctx, const Job& job, uint64_t n) {
  std::lock_guard<std::mutex> lock(ctx->mu);
  const size_t nw = ctx->workers.size();
  if (nw == 1 || n < 2 * nw) return worker_run(ctx->workers[0], job, 0, n);
  std::vector<int> rcs(nw, LBF_OK);
  std::vector<std::string> errs(nw);
  std::vector<std::thread> th;
  for (size_t d = 0; d < nw; ++d) {
    const uint64_t b = n * d / nw, e = n * (d + 1) / nw;
    th.emplace_back([&, d, b, e] {
      rcs[d] = worker_run(ctx->workers[d], job, b, e);
      if (rcs[d]) errs[d] = lbf_last_error();
    });
  }
  for (auto& t : th) t.join();
  for (size_t d = 0; d < nw; ++d)
    if (rcs[d]) return fail(rcs[d], "device " + std::to_string(ctx->workers[d].device) + ": " + errs[d]);
  return LBF_OK;
}

// Device-pointer batch: synchronous on worker 0's first stream.
int run_device_job(lbf_ctx* ctx, const uint8_t* base, const uint64_t* offsets, const uint32_t* sizes,
                   uint64_t n, uint8_t* digests, const uint8_t* expected, uint8_t* verdicts) {
  std::lock_guard<std::mutex> lock(ctx->mu);
  Worker& w = ctx->workers[0];
  LBF_HIP_TRY(hipSetDevice(w.device));
  hipStream_t s = w.slot[0].stream;
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

extern "C" int lbf_ctx_create(uint32_t device_mask, lbf_ctx** out) {
  if (!out) return fail(LBF_ERR_INVALID, "null out");
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return fail(LBF_ERR_NO_DEVICE, "no GPU visible: the chunk-hash path runs only on MI355X (no CPU fallback)");
  lbf_ctx* ctx = new lbf_ctx();
  for (int d = 0; d < ndev && d < 32; ++d) {
    if (device_mask && !(device_mask & (1u << d))) continue;
    ctx->workers.emplace_back();
    if (int rc = worker_init(ctx->workers.back(), d)) {
      std::string msg = lbf_last_error();
      lbf_ctx_destroy(ctx);
      return fail(rc, msg);
    }
  }
  if (ctx->workers.empty()) {
    delete ctx;
    return fail(LBF_ERR_NO_DEVICE, "device_mask selects no visible device");
  }
  *out = ctx;
  return LBF_OK;
}

extern "C" void lbf_ctx_destroy(lbf_ctx* ctx) {
  if (!ctx) return;
  for (Worker& w : ctx->workers) worker_free(w);
  delete ctx;
}

extern "C" int lbf_ctx_num_devices(const lbf_ctx* ctx) { return ctx ? (int)ctx->workers.size() : 0; }

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
  return run_job(ctx, job, n);
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
  return run_job(ctx, job, n);
}

extern "C" int lbf_file_ranges(lbf_ctx* ctx, const char* path, const uint64_t* offsets, const uint32_t* sizes,
                               uint64_t n, const uint8_t* expected, uint8_t* out) {
  if (!ctx || !path) return fail(LBF_ERR_INVALID, "null context/path");
  if (n == 0) return LBF_OK;
  if (!offsets || !sizes || !out) return fail(LBF_ERR_INVALID, "null argument");
  const int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) {
    if (!expected) return fail(LBF_ERR_IO, std::string("cannot open ") + path);
    memset(out, 0, n);  // Flood.cpp:257: no file -> every chunk stays '0'
    return LBF_OK;
  }
  posix_fadvise(fd, 0, 0, POSIX_FADV_SEQUENTIAL);
  Job job{};
  job.src.fd = fd;
  job.offsets = offsets;
  job.sizes = sizes;
  job.expected = expected;
  if (expected) job.verdicts = out;
  else job.digests = out;
  const int rc = run_job(ctx, job, n);
  close(fd);
  return rc;
}

extern "C" int lbf_sha1_one(lbf_ctx* ctx, const uint8_t* data, uint32_t size, uint8_t out[20]) {
  static const uint8_t kEmpty = 0;
  if (!data && size) return fail(LBF_ERR_INVALID, "null data");
  const uint64_t off = 0;
  return lbf_sha1_batch(ctx, data ? data : &kEmpty, size, &off, &size, 1, out, LBF_HOST_PTR);
}
