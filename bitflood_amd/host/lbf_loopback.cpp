// lbf_loopback.cpp -- configuration C5: two peers over loopback TCP, every
// received chunk verified on the GPU before it is written.
//
// Seeder  : a test_client that holds the whole file.  For RequestChunk it reads
//           the chunk, re-verifies it and answers SendChunk only if it matches
//           (ChunkMethodHandler::_HandleRequestChunk, ChunkMethods.cpp:89-135).
// Leecher : a test_client that holds nothing.  It asks for chunks
//           (Flood::LoopOnce, Flood.cpp:85-165) and handles SendChunk by size
//           check, verify, write at the chunk's offset, chunkmap '1'
//           (_HandleSendChunk, ChunkMethods.cpp:137-225).
// Both speak the reference's frames (include/libBitFlood/PeerWire.H).
//
// What differs from the reference loop, on purpose:
//  - no tracker: the leecher connects to the seeder directly (registration is
//    control plane, out of scope);
//  - no pacing: the reference sleeps 100 ms per loop and asks for one chunk per
//    loop (test_client.cpp:72-76, Flood.cpp:95-141), about 10 chunks/s.  Here the
//    leecher keeps --window requests outstanding;
//  - batched verify: up to --batch arrivals per GPU launch (Flood::ReceiveChunks)
//    and up to --batch requests per launch on the seeder (ReadVerifiedChunks).
//    While a verify runs, the next batch starts when it is full or when its
//    oldest arrival has waited --deadline-ms (default 10; 0 = only when full),
//    which bounds the verify latency the batching adds.
// With --corrupt K the seeder flips one byte of every K-th chunk AFTER its own
// verify (a wire error); the leecher must reject it and ask again.
// With --synthetic the seeder holds no file: its chunk bytes come from the
// counter-mode generator (the stream lbf_fill_synthetic writes), re-verified on
// the GPU against the flood file before sending (Flood::VerifyChunks, the verify
// half of _HandleRequestChunk), and the flood file is encoded from the same
// stream generated in HBM.  Only the leecher's copy touches the disk, so the
// 16 GiB C5 transfer needs 16 GiB of scratch space, not 32; the written file is
// compared with the generator instead of a source file.
//
// Prints one JSON line: payload rate, verify latency (frame arrival -> GPU
// verdict) and accept latency (arrival -> chunk written), batch sizes, and the end
// state (resume verify of the written file, byte comparison with the source).
//
// Process shape (--role).  The reference's peers are separate OS processes, two
// test_client runs (test_client.cpp:27-77) on one box, each with its own select
// loop.  --role seeder and --role leecher are those two
// processes: each owns its HIP runtime, its GPU contexts, its arenas and their
// registrations, and neither sees the other's.  The seeder writes the flood file
// (test_encoder's part) into --dir, listens on 127.0.0.1 (--port, 0 = any) and
// writes the port to --port-file once it is listening; the leecher loads the
// flood file from --dir and connects to --port.  Each prints its own JSON line
// (tests/test_host_cpp.py merges them).  The default, --role both, runs the two
// peers as threads of one process, the round-1 to round-4 harness.
#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/statvfs.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "lbf_hash.h"
#include "libBitFlood/Encoder.H"
#include "libBitFlood/Flood.H"
#include "libBitFlood/FloodFile.H"
#include "libBitFlood/PeerWire.H"

using namespace libBitFlood;
using Clock = std::chrono::steady_clock;

namespace {

struct Opts {
  U64 size = 256ull << 20;
  U32 chunksize = 262144;
  U32 window = 512;
  U32 batch = 128;
  U32 deadline_ms = 10;  // flush a partial batch once its oldest arrival waited this long
  unsigned threads = 8;
  U32 corrupt = 0;
  std::string dir;
  bool keep = false;
  bool synthetic = false;
  bool register_arenas = true;  // --no-register: stage the leecher's verifies (A/B)
  unsigned verifiers = 2;        // leecher: GPU verifies in flight (each its own context)
  bool seeder_pipeline = false;  // --pipelined-seeder: verify batch k+1 while batch k is encoded
  bool gpu_decode = true;        // the leecher's base64 decode on the GPU with its verify (--cpu-decode: on the host)
  bool gpu_encode = false;       // --gpu-encode: the seeder's base64 encode on the GPU with its verify (--synthetic)
  unsigned seeder_workers = 1;   // --seeder-workers S: the seeder's verify/encode workers (each its own context)
  enum Role { BOTH, SEEDER, LEECHER } role = BOTH;  // --role: both peers in this process, or one of them
  int port = -1;                 // seeder: port to listen on (0 / unset = any); leecher: port to dial
  std::string port_file;         // seeder: where to write the port once listening
};

[[noreturn]] void die(const std::string& m) {
  fprintf(stderr, "lbf_loopback: %s\n", m.c_str());
  exit(2);
}

double secs(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

// A pool of threads kept for the whole transfer: each batch's decode (leecher)
// and generate / encode (seeder) runs over it.  Starting and joining sixteen
// threads per batch, as parallel_for does, cost ~0.7 ms of every ~40-chunk
// batch's latency.  run() hands out indices through an atomic counter; the
// calling thread works too and returns once every index is done.
class Pool {
 public:
  explicit Pool(unsigned threads) {
    for (unsigned t = 1; t < threads; ++t) th_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (std::thread& t : th_) t.join();
  }
  template <class F>
  void run(size_t n, F&& f) {
    if (n <= 1 || th_.empty()) {
      for (size_t k = 0; k < n; ++k) f(k);
      return;
    }
    std::function<void(size_t)> fn(std::forward<F>(f));
    {
      std::lock_guard<std::mutex> g(mu_);
      job_ = &fn;
      n_ = n;
      next_ = 0;
      busy_ = th_.size();
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> g(mu_);
    done_.wait(g, [&] { return busy_ == 0; });
    job_ = nullptr;
  }

 private:
  void work() {
    for (size_t k; (k = next_++) < n_;) (*job_)(k);
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
      }
      work();
      std::lock_guard<std::mutex> g(mu_);
      if (--busy_ == 0) done_.notify_one();
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  std::function<void(size_t)>* job_ = nullptr;
  std::atomic<size_t> next_{0};
  size_t n_ = 0, busy_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

template <class F>
void parallel_for(size_t n, unsigned threads, F f) {
  if (n <= 1 || threads <= 1) {
    for (size_t k = 0; k < n; ++k) f(k);
    return;
  }
  std::atomic<size_t> next{0};
  std::vector<std::thread> th;
  for (unsigned t = 0; t < std::min<size_t>(threads, n); ++t)
    th.emplace_back([&] {
      for (size_t k; (k = next++) < n;) f(k);
    });
  for (auto& t : th) t.join();
}

// ---- sockets ---------------------------------------------------------------
void tune(int fd) {
  int one = 1, buf = 8 << 20;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof(buf));
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof(buf));
}

int listen_loopback(int& port) {
  const int fd = socket(AF_INET, SOCK_STREAM, 0);
  if (fd < 0) die("socket failed");
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  a.sin_port = htons((uint16_t)(port > 0 ? port : 0));
  if (bind(fd, (sockaddr*)&a, sizeof(a)) != 0 || listen(fd, 1) != 0) die("bind/listen on 127.0.0.1 failed");
  socklen_t len = sizeof(a);
  getsockname(fd, (sockaddr*)&a, &len);
  port = ntohs(a.sin_port);
  return fd;
}

int connect_loopback(int port) {
  const int fd = socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  a.sin_port = htons((uint16_t)port);
  if (fd < 0 || connect(fd, (sockaddr*)&a, sizeof(a)) != 0) die("connect to 127.0.0.1 failed");
  tune(fd);
  return fd;
}

bool send_all(int fd, const std::string& s) {
  size_t put = 0;
  while (put < s.size()) {
    const ssize_t w = send(fd, s.data() + put, s.size() - put, MSG_NOSIGNAL);
    if (w <= 0) return false;
    put += (size_t)w;
  }
  return true;
}

// '\n'-delimited frames (PeerConnection.cpp:213-237).
struct FrameReader {
  explicit FrameReader(int f) : fd(f) {}
  int fd;
  std::string buf;
  size_t head = 0, scan = 0;
  bool buffered() {
    return memchr(buf.data() + scan, '\n', buf.size() - scan) != nullptr;
  }
  bool next(std::string& frame) {
    for (;;) {
      const char* nl = (const char*)memchr(buf.data() + scan, '\n', buf.size() - scan);
      if (nl) {
        const size_t end = (size_t)(nl - buf.data());
        frame.assign(buf.data() + head, end - head);
        head = scan = end + 1;
        if (head > (64u << 20)) {  // compact
          buf.erase(0, head);
          head = scan = 0;
        }
        return true;
      }
      scan = buf.size();
      const size_t old = buf.size();
      buf.resize(old + (4 << 20));
      const ssize_t r = recv(fd, &buf[old], 4 << 20, 0);
      buf.resize(old + (r > 0 ? (size_t)r : 0));
      if (r <= 0) return false;
    }
  }
};

// ---- synthetic source file -------------------------------------------------
// Counter-mode splitmix64, the same stream as the device fill (sha1_device.hpp).
U64 synth_word(U64 seed, U64 k) {
  U64 z = seed * 0xD1B54A32D192ED03ull + (k + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void write_source(const std::string& path, U64 size, unsigned threads) {
  const int fd = open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) die("cannot create " + path);
  const U64 block = 64ull << 20;
  const U64 nblk = (size + block - 1) / block;
  std::atomic<bool> ok{true};
  parallel_for(nblk, threads, [&](size_t b) {
    const U64 off = b * block, len = std::min(block, size - off);
    std::vector<U64> w((len + 7) / 8);
    for (U64 k = 0; k < w.size(); ++k) w[k] = synth_word(0xC5, off / 8 + k);
    if (pwrite(fd, w.data(), len, (off_t)off) != (ssize_t)len) ok = false;
  });
  close(fd);
  if (!ok) die("writing " + path + " failed");
}

constexpr U64 kSeed = 0xC5;

// Bytes [off, off + len) of the synthetic stream.
void synth_bytes(U8* dst, U64 off, U64 len) {
  U64 k = off / 8, pos = off;
  const U64 end = off + len;
  if (pos % 8) {  // leading partial word
    const U64 w = synth_word(kSeed, k++);
    for (; pos < end && pos % 8; ++pos) *dst++ = (U8)(w >> (8 * (pos % 8)));
  }
  for (; pos + 8 <= end; pos += 8, dst += 8) {
    const U64 w = synth_word(kSeed, k++);
    memcpy(dst, &w, 8);
  }
  if (pos < end) {
    const U64 w = synth_word(kSeed, k);
    for (U64 b = 0; pos < end; ++pos, ++b) *dst++ = (U8)(w >> (8 * b));
  }
}

// The flood file of the synthetic stream, hashed where it is generated: in HBM
// (lbf_fill_synthetic + one device-resident batch launch), like test_encoder
// run over the seeder's file.
void encode_synthetic(const std::string& name, U64 size, U32 cs, FloodFile& ff) {
  const U64 n = (size + cs - 1) / cs;
  FloodFile::FileSPtr file(new FloodFile::File());
  file->m_name = name;
  file->m_size = size;
  file->m_chunks.resize(n);
  if (n) {
    void *d_buf = nullptr, *d_dig = nullptr;
    if (lbf_dev_malloc(&d_buf, size) != LBF_OK || lbf_dev_malloc(&d_dig, n * 20) != LBF_OK ||
        lbf_fill_synthetic((U8*)d_buf, size, kSeed, 0, nullptr) != LBF_OK ||
        lbf_sha1_uniform_launch((const U8*)d_buf, size, cs, 0, n, (U8*)d_dig, nullptr, nullptr, nullptr) != LBF_OK ||
        lbf_device_synchronize() != LBF_OK)
      die(std::string("synthetic encode failed: ") + lbf_last_error());
    V_U8 dig(n * 20);
    if (lbf_memcpy_d2h(dig.data(), d_dig, n * 20) != LBF_OK) die(std::string("D2H failed: ") + lbf_last_error());
    lbf_dev_free(d_buf);
    lbf_dev_free(d_dig);
    for (U64 i = 0; i < n; ++i) {
      FloodFile::Chunk& c = file->m_chunks[i];
      c.m_index = (U32)i;
      c.m_size = (U32)std::min<U64>(cs, size - i * cs);
      c.m_weight = 0;
      char b64[28];
      lbf_b64_27(&dig[20 * i], b64);
      c.m_hash.assign(b64, 27);
    }
  }
  ff.m_files[name] = file;
}

// The leecher's file equals the synthetic stream (a missing file equals an
// empty stream: the leecher creates its file on the first chunk it accepts).
bool file_matches_synthetic(const std::string& path, U64 size, unsigned threads) {
  struct stat st;
  if (stat(path.c_str(), &st) != 0) return size == 0;
  if ((U64)st.st_size != size) return false;
  const int fd = open(path.c_str(), O_RDONLY);
  if (fd < 0) return false;
  const U64 block = 64ull << 20;
  std::atomic<bool> eq{true};
  parallel_for((size + block - 1) / block, threads, [&](size_t b) {
    const U64 off = b * block, len = std::min(block, size - off);
    V_U8 got(len), want(len);
    if (pread(fd, got.data(), len, (off_t)off) != (ssize_t)len) eq = false;
    synth_bytes(want.data(), off, len);
    if (memcmp(got.data(), want.data(), len) != 0) eq = false;
  });
  close(fd);
  return eq;
}

// The leecher creates a file on its first received chunk (ChunkMethods.cpp:169-172),
// so a zero-chunk (empty) file is never created: an empty seed file and a missing
// leech file count as equal, as they would for the reference's peers.
bool files_equal(const std::string& a, const std::string& b) {
  FILE* fa = fopen(a.c_str(), "rb");
  FILE* fb = fopen(b.c_str(), "rb");
  if (fa && !fb) {
    const bool empty = fgetc(fa) == EOF;
    fclose(fa);
    return empty;
  }
  bool eq = fa && fb;
  std::vector<char> x(16 << 20), y(16 << 20);
  while (eq) {
    const size_t ra = fread(x.data(), 1, x.size(), fa), rb = fread(y.data(), 1, y.size(), fb);
    if (ra != rb || memcmp(x.data(), y.data(), ra) != 0) eq = false;
    if (ra < x.size()) break;
  }
  if (fa) fclose(fa);
  if (fb) fclose(fb);
  return eq;
}

// ---- seeder ------------------------------------------------------------------
struct SeederStats {
  U64 requests = 0, sent = 0, refused = 0, corrupted = 0;
  double verify_s = 0, encode_s = 0;
};

// Blocking queue (closing wakes every waiter).
template <class T>
struct Chan {
  std::mutex mu;
  std::condition_variable cv;
  std::deque<T> q;
  bool closed = false;
  void put(T v) {
    std::lock_guard<std::mutex> g(mu);
    q.push_back(std::move(v));
    cv.notify_all();
  }
  void close() {
    std::lock_guard<std::mutex> g(mu);
    closed = true;
    cv.notify_all();
  }
  // up to `max` items; blocks for the first; false once closed and drained
  bool take(std::vector<T>& out, size_t max) {
    out.clear();
    std::unique_lock<std::mutex> g(mu);
    cv.wait(g, [&] { return !q.empty() || closed; });
    while (!q.empty() && out.size() < max) {
      out.push_back(std::move(q.front()));
      q.pop_front();
    }
    return !out.empty();
  }
};

// Seeder pipeline: reader thread (frames -> request keys), S workers (read +
// GPU verify + parallel encode of a batch; each its own GPU context, arenas and
// thread pool, taking whatever requests are queued when it is free), sender
// thread (frames -> socket).  A batch costs at least one chunk's SHA-1 chain on
// the GPU (3.1 ms at 256 KiB) however few chains it holds, so a second worker
// verifies the next requests while the first waits for its chain.
// --pipelined-seeder moves each worker's encode to a thread of its own, so batch
// k+1 is read and verified while batch k is encoded.  On the 16-CPU GPU box that
// did not raise the transfer rate and cost latency: the generator and the
// encoder then compete for the same cores, so it is not the
// default.
void seeder_main(int lfd, FloodFileSPtr ff, std::string root, const Opts& o, SeederStats& st) {
  // a seeder process whose leecher never comes must still end
  pollfd pl{lfd, POLLIN, 0};
  if (poll(&pl, 1, 300 * 1000) != 1) die("seeder: no leecher connected within 300 s");
  const int fd = accept(lfd, nullptr, nullptr);
  if (fd < 0) die("accept failed");
  tune(fd);
  // the seeder is its own peer: its own GPU contexts (streams, staging), one per
  // worker, and one resume verify whose result every worker copies
  std::vector<lbf_ctx*> wctx(o.seeder_workers, nullptr);
  for (unsigned w = 0; w < o.seeder_workers; ++w)
    if (lbf_ctx_create(0, &wctx[w]) != LBF_OK) die(std::string("seeder: lbf_ctx_create: ") + lbf_last_error());
  Flood fl0;
  fl0.m_rootdir = root;
  fl0.m_ctx = wctx[0];
  if (fl0.Initialize(ff) != Error::NO_ERROR_LBF) die("seeder: Initialize failed: " + std::string(Encoder::LastError()));
  Chan<Flood::P_ChunkKey> requests;
  Chan<std::string> outbox;
  std::thread reader([&] {
    FrameReader rd(fd);
    std::string f, method;
    std::vector<PeerWire::Value> params;
    while (rd.next(f))
      if (PeerWire::DecodeMethod(f, method, params) && method == PeerWire::kRequestChunk && params.size() == 2 &&
          params[0].m_type == PeerWire::Value::STRING && params[1].m_type == PeerWire::Value::INT)
        requests.put(Flood::P_ChunkKey(params[0].m_str, (U32)params[1].m_int));
    requests.close();
  });
  std::thread sender([&] {
    std::vector<std::string> msgs;
    bool ok = true;
    while (outbox.take(msgs, 64))
      for (const std::string& m : msgs) ok = ok && send_all(fd, m);
  });
  std::mutex shared_mu;          // the workers' shared state below
  Flood::S_ChunkKey corrupted;   // chunks already sent corrupted once
  const U64 page = (U64)sysconf(_SC_PAGESIZE);
  const U64 slot_bytes = ((U64)o.chunksize + 15) & ~15ull;
  const U64 synth_cap = (slot_bytes * o.batch + page - 1) / page * page;
  // --gpu-encode: each arena's chunks come back from the GPU as base64 text,
  // one 16-byte aligned slot per chunk, in a text arena of its own
  const U64 text_slot = (PeerWire::Base64PutLength(o.chunksize) + 15) & ~15ull;
  const U64 text_cap = o.gpu_encode ? (text_slot * o.batch + page - 1) / page * page : 0;
  const unsigned pool_threads = std::max(1u, o.threads / o.seeder_workers);
  auto worker = [&](unsigned w) {
    lbf_ctx* ctx = wctx[w];
    Flood fl;
    fl.m_floodfile = fl0.m_floodfile;
    fl.m_runtimefiles = fl0.m_runtimefiles;
    fl.m_rootdir = fl0.m_rootdir;
    fl.m_ctx = ctx;
    SeederStats mine;
    // Two arenas per worker (one being verified, one being encoded),
    // page-aligned and (unless --no-register) registered with the worker's
    // context, like the leecher's: a batch costs no allocation, no zero fill of
    // up to batch x chunk bytes, and no staging copy on its verify.
    // ReadVerifiedChunks keeps its own vectors the same way.
    constexpr int kSeedArenas = 2;
    U8* synth_mem = nullptr;
    if (o.synthetic) {
      synth_mem = static_cast<U8*>(aligned_alloc(page, synth_cap * kSeedArenas));
      if (!synth_mem) die("seeder: cannot allocate the arenas");
      memset(synth_mem, 0, synth_cap * kSeedArenas);
      for (int a = 0; a < kSeedArenas; ++a)
        if (o.register_arenas && lbf_host_register(ctx, synth_mem + a * synth_cap, synth_cap) != LBF_OK)
          die("seeder: lbf_host_register failed: " + std::string(lbf_last_error()));
    }
    char* text_mem = nullptr;
    if (o.gpu_encode) {
      text_mem = static_cast<char*>(aligned_alloc(page, text_cap * kSeedArenas));
      if (!text_mem) die("seeder: cannot allocate the text arenas");
      memset(text_mem, 0, text_cap * kSeedArenas);
      for (int a = 0; a < kSeedArenas; ++a)
        if (o.register_arenas && lbf_host_register(ctx, text_mem + a * text_cap, text_cap) != LBF_OK)
          die("seeder: lbf_host_register failed: " + std::string(lbf_last_error()));
    }
    V_U8 file_arena[kSeedArenas];
    Pool gen_pool(pool_threads);                                        // this worker's generate
    std::unique_ptr<Pool> enc_pool_own(o.seeder_pipeline ? new Pool(pool_threads) : nullptr);
    Pool& enc_pool = o.seeder_pipeline ? *enc_pool_own : gen_pool;  // the encode stage's
    struct Verified {
      std::vector<Flood::P_ChunkKey> keys;
      V_U64 offs;
      V_U64 toffs;  // --gpu-encode: the text slots
      std::string valid;
      int arena = 0;
    };
    Chan<Verified> to_encode;
    Chan<int> free_arena;
    for (int a = 0; a < kSeedArenas; ++a) free_arena.put(a);
    auto encode = [&](Verified& v) {
      const std::vector<Flood::P_ChunkKey>& keys = v.keys;
      const U8* arena = o.synthetic ? synth_mem + v.arena * synth_cap : file_arena[v.arena].data();
      auto t1 = Clock::now();
      // sizes and the (first-send-only) corruption decision, serially
      std::vector<U32> sizes(keys.size(), 0);
      std::vector<char> flip(keys.size(), 0);
      {
        std::lock_guard<std::mutex> g(shared_mu);
        for (size_t k = 0; k < keys.size(); ++k) {
          if (v.valid[k] != '1') continue;
          sizes[k] = fl.m_runtimefiles.find(keys[k].first)->second.m_file->m_chunks[keys[k].second].m_size;
          if (o.corrupt && sizes[k] && keys[k].second % o.corrupt == o.corrupt - 1 &&
              corrupted.insert(keys[k]).second) {
            flip[k] = 1;
            ++mine.corrupted;
          }
        }
      }
      std::vector<std::string> out(keys.size());
      enc_pool.run(keys.size(), [&](size_t k) {
        if (v.valid[k] != '1') return;  // "send only if equal" (ChunkMethods.cpp:117-123)
        if (o.gpu_encode) {  // the GPU's text; a wire error flips one of its characters
          const char* t = text_mem + v.arena * text_cap + v.toffs[k];
          const size_t tl = PeerWire::Base64PutLength(sizes[k]);
          if (!flip[k]) {
            out[k] = PeerWire::FrameSendChunkText(keys[k].first, keys[k].second, t, tl);
            return;
          }
          std::string tmp(t, tl);
          const size_t g = sizes[k] / 2 / 3, at = 4 * g + g / 18;  // a character of the middle byte's group
          tmp[at] = tmp[at] == 'A' ? 'B' : 'A';
          out[k] = PeerWire::FrameSendChunkText(keys[k].first, keys[k].second, tmp.data(), tl);
          return;
        }
        const U8* data = arena + v.offs[k];
        std::vector<U8> tmp;
        if (flip[k]) {  // a wire error after the seeder's own verify
          tmp.assign(data, data + sizes[k]);
          tmp[sizes[k] / 2] ^= 0x01;
          data = tmp.data();
        }
        out[k] = PeerWire::EncodeSendChunk(keys[k].first, keys[k].second, data, sizes[k]);
      });
      mine.encode_s += secs(t1, Clock::now());
      for (std::string& m : out) {
        if (m.empty()) {
          ++mine.refused;
          continue;
        }
        ++mine.sent;
        outbox.put(std::move(m));
      }
    };
    std::thread encoder;
    if (o.seeder_pipeline)
      encoder = std::thread([&] {
        std::vector<Verified> vs;
        while (to_encode.take(vs, 1)) {
          encode(vs[0]);
          free_arena.put(vs[0].arena);
        }
      });
    std::vector<Flood::P_ChunkKey> keys;
    std::vector<int> ar;
    while (requests.take(keys, o.batch)) {
      mine.requests += keys.size();
      if (!free_arena.take(ar, 1)) break;
      Verified v;
      v.arena = ar[0];
      auto t0 = Clock::now();
      if (o.synthetic) {
        // the requested chunks from the generator, 16-byte aligned in the arena,
        // then the same GPU re-verify before sending (ChunkMethods.cpp:116-123)
        U8* arena = synth_mem + v.arena * synth_cap;
        std::vector<Flood::ChunkArrival> chunks(keys.size());
        v.offs.assign(keys.size(), 0);
        U64 total = 0;
        for (size_t k = 0; k < keys.size(); ++k) {
          auto it = fl.m_runtimefiles.find(keys[k].first);
          U32 sz = 0;
          if (it != fl.m_runtimefiles.end() && keys[k].second < it->second.m_file->m_chunks.size())
            sz = it->second.m_file->m_chunks[keys[k].second].m_size;
          v.offs[k] = total;
          chunks[k] = Flood::ChunkArrival{keys[k].first, keys[k].second, total, sz};
          total += (sz + 15) & ~15ull;
        }
        if (total > synth_cap) die("seeder: batch larger than its arena");
        gen_pool.run(keys.size(), [&](size_t k) {
          auto it = fl.m_runtimefiles.find(keys[k].first);
          if (chunks[k].m_size == 0 || it == fl.m_runtimefiles.end()) return;
          synth_bytes(arena + v.offs[k], it->second.m_chunkoffsets[keys[k].second], chunks[k].m_size);
        });
        if (o.gpu_encode) {
          v.toffs.resize(keys.size());
          for (size_t k = 0; k < keys.size(); ++k) v.toffs[k] = k * text_slot;
          if (fl.VerifyEncodeChunks(arena, synth_cap, chunks, v.valid, text_mem + v.arena * text_cap, text_cap,
                                    v.toffs) != Error::NO_ERROR_LBF)
            die("seeder: verify + encode failed: " + std::string(Encoder::LastError()));
        } else if (fl.VerifyChunks(arena, synth_cap, chunks, v.valid) != Error::NO_ERROR_LBF) {
          die("seeder: verify failed: " + std::string(Encoder::LastError()));
        }
      } else if (fl.ReadVerifiedChunks(keys, file_arena[v.arena], v.offs, v.valid) != Error::NO_ERROR_LBF) {
        die("seeder: verify failed: " + std::string(Encoder::LastError()));
      }
      mine.verify_s += secs(t0, Clock::now());
      v.keys = std::move(keys);
      keys = std::vector<Flood::P_ChunkKey>();
      if (o.seeder_pipeline) {
        to_encode.put(std::move(v));
      } else {
        encode(v);
        free_arena.put(v.arena);
      }
    }
    to_encode.close();
    if (encoder.joinable()) encoder.join();
    if (synth_mem) {
      for (int a = 0; a < kSeedArenas; ++a)
        if (o.register_arenas) (void)lbf_host_unregister(ctx, synth_mem + a * synth_cap);
      free(synth_mem);
    }
    if (text_mem) {
      for (int a = 0; a < kSeedArenas; ++a)
        if (o.register_arenas) (void)lbf_host_unregister(ctx, text_mem + a * text_cap);
      free(text_mem);
    }
    std::lock_guard<std::mutex> g(shared_mu);
    st.requests += mine.requests;
    st.sent += mine.sent;
    st.refused += mine.refused;
    st.corrupted += mine.corrupted;
    st.verify_s += mine.verify_s;
    st.encode_s += mine.encode_s;
  };
  std::vector<std::thread> others;
  for (unsigned w = 1; w < o.seeder_workers; ++w) others.emplace_back(worker, w);
  worker(0);
  for (std::thread& t : others) t.join();
  outbox.close();
  sender.join();
  reader.join();
  close(fd);
  for (lbf_ctx* c : wctx) lbf_ctx_destroy(c);
}

// ---- leecher -------------------------------------------------------------------
struct Arrival {
  std::string frame;
  Clock::time_point t;
};


}  // namespace

int main(int argc, char** argv) {
  Opts o;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto val = [&]() -> const char* {
      if (i + 1 >= argc) die("missing value for " + a);
      return argv[++i];
    };
    if (a == "--size") o.size = strtoull(val(), nullptr, 10);
    else if (a == "--chunksize") o.chunksize = (U32)strtoul(val(), nullptr, 10);
    else if (a == "--window") o.window = (U32)strtoul(val(), nullptr, 10);
    else if (a == "--batch") o.batch = (U32)strtoul(val(), nullptr, 10);
    else if (a == "--deadline-ms") o.deadline_ms = (U32)strtoul(val(), nullptr, 10);
    else if (a == "--threads") o.threads = (unsigned)strtoul(val(), nullptr, 10);
    else if (a == "--corrupt") o.corrupt = (U32)strtoul(val(), nullptr, 10);
    else if (a == "--dir") o.dir = val();
    else if (a == "--keep") o.keep = true;
    else if (a == "--synthetic") o.synthetic = true;
    else if (a == "--no-register") o.register_arenas = false;
    else if (a == "--verifiers") o.verifiers = (unsigned)strtoul(val(), nullptr, 10);
    else if (a == "--pipelined-seeder") o.seeder_pipeline = true;
    else if (a == "--gpu-decode") o.gpu_decode = true;
    else if (a == "--cpu-decode") o.gpu_decode = false;
    else if (a == "--seeder-workers") o.seeder_workers = (unsigned)strtoul(val(), nullptr, 10);
    else if (a == "--gpu-encode") o.gpu_encode = true;
    else if (a == "--cpu-encode") o.gpu_encode = false;
    else if (a == "--role") {
      const std::string r = val();
      if (r == "both") o.role = Opts::BOTH;
      else if (r == "seeder") o.role = Opts::SEEDER;
      else if (r == "leecher") o.role = Opts::LEECHER;
      else die("--role takes both, seeder or leecher");
    } else if (a == "--port") {
      const long v = strtol(val(), nullptr, 10);
      if (v < 0 || v > 65535) die("--port must be 0..65535");
      o.port = (int)v;
    }
    else if (a == "--port-file") o.port_file = val();
    else {
      fprintf(stderr,
              "usage: lbf_loopback [--size BYTES] [--chunksize N] [--window W] [--batch B] [--deadline-ms MS]\n"
              "                    [--threads T]\n"
              "                    [--corrupt K] [--dir DIR] [--keep] [--synthetic] [--no-register]\n"
              "                    [--verifiers V] [--pipelined-seeder] [--gpu-decode | --cpu-decode]\n"
              "                    [--gpu-encode | --cpu-encode] [--seeder-workers S]\n"
              "                    [--role both | --role seeder [--port P] [--port-file F] |\n"
              "                     --role leecher --port P]   (seeder and leecher: same --dir and options)\n");
      return 2;
    }
  }
  if (o.chunksize == 0 || o.window == 0 || o.batch == 0) die("chunksize, window and batch must be > 0");
  if (o.verifiers == 0 || o.verifiers > 8) die("verifiers must be 1..8");
  if (o.seeder_workers == 0 || o.seeder_workers > 8) die("seeder workers must be 1..8");
  if (o.gpu_encode && !o.synthetic) die("--gpu-encode needs --synthetic (the file seeder reads and verifies in one call)");
  if (o.role != Opts::BOTH && o.dir.empty()) die("--role seeder/leecher needs --dir (the directory both peers share)");
  if (o.role == Opts::LEECHER && (o.port <= 0 || o.port > 65535)) die("--role leecher needs --port");
  if (o.dir.empty()) {
    const char* t = getenv("TMPDIR");
    char tmpl[512];
    snprintf(tmpl, sizeof(tmpl), "%s/lbf_loopback.XXXXXX", t && *t ? t : "/tmp");
    if (!mkdtemp(tmpl)) die("mkdtemp failed");
    o.dir = tmpl;
  }
  const bool is_seeder = o.role != Opts::LEECHER, is_leecher = o.role != Opts::SEEDER;
  const std::string seeddir = o.dir + "/seed", leechdir = o.dir + "/leech";
  mkdir(o.dir.c_str(), 0755);
  if (is_seeder) mkdir(seeddir.c_str(), 0755);
  if (is_leecher) mkdir(leechdir.c_str(), 0755);
  struct statvfs vfs;
  // the bytes this process writes: the seeder's file (not with --synthetic), the leecher's copy
  const U64 copies = (is_seeder && !o.synthetic ? 1 : 0) + (is_leecher ? 1 : 0);
  if (statvfs(o.dir.c_str(), &vfs) == 0 && (U64)vfs.f_bavail * vfs.f_frsize < copies * o.size + (64 << 20))
    die("not enough free space in " + o.dir + " for " + std::to_string(copies) + " copies of the file");

  // The seeder's file and the flood file both peers load (test_encoder + test_client).
  const std::string name = "c5.bin";
  const std::string floodpath = o.dir + "/c5.flood";
  double encode_s = 0;
  FloodFileSPtr ff(new FloodFile());
  if (is_seeder) {
    FloodFile encoded;
    auto te0 = Clock::now();
    if (o.synthetic) {
      encode_synthetic(seeddir + "/" + name, o.size, o.chunksize, encoded);
    } else {
      write_source(seeddir + "/" + name, o.size, o.threads);
      te0 = Clock::now();
      Encoder::ToEncode te;
      te.m_files.push_back(seeddir + "/" + name);
      te.m_chunksize = o.chunksize;
      if (Encoder::EncodeFile(te, encoded) != Error::NO_ERROR_LBF)
        die("EncodeFile failed: " + std::string(Encoder::LastError()));
    }
    encode_s = secs(te0, Clock::now());
    // peers address the file by its name relative to their own directory
    for (auto& kv : encoded.m_files) {
      FloodFile::FileSPtr file = kv.second;
      file->m_name = name;
      ff->m_files[name] = file;
    }
    if (ff->ToXMLFile(floodpath) != Error::NO_ERROR_LBF) die("ToXMLFile failed");
  }

  int port = o.port > 0 ? o.port : 0;
  const int lfd = is_seeder ? listen_loopback(port) : -1;
  SeederStats sst;
  if (o.role == Opts::SEEDER) {
    // The flood file is complete before the port is published, so a leecher
    // started on the port file finds it.  Written then renamed: never half a number.
    if (!o.port_file.empty()) {
      const std::string tmp = o.port_file + ".tmp";
      FILE* pf = fopen(tmp.c_str(), "w");
      if (!pf || fprintf(pf, "%d\n", port) < 0 || fclose(pf) != 0 || rename(tmp.c_str(), o.port_file.c_str()) != 0)
        die("cannot write the port file " + o.port_file);
    }
    fprintf(stderr, "lbf_loopback: seeder listening on 127.0.0.1:%d\n", port);
    const auto s0 = Clock::now();
    seeder_main(lfd, ff, seeddir, o, sst);
    const double serve_s = secs(s0, Clock::now());
    close(lfd);
    printf("{\"config\": \"C5 loopback 2-peer\", \"role\": \"seeder\", \"pid\": %d, \"bytes\": %llu, "
           "\"chunk_size\": %u, \"chunks\": %zu, \"batch\": %u, \"seeder_pipelined\": %s, \"gpu_encode\": %s, "
           "\"seeder_workers\": %u, \"threads\": %u, \"seconds\": %.3f, \"encode_flood_s\": %.3f, "
           "\"seeder\": {\"requests\": %llu, \"sent\": %llu, \"refused\": %llu, \"verify_s\": %.3f, "
           "\"encode_s\": %.3f}, \"corrupt_every\": %u, \"corrupted_sent\": %llu, \"seed_source\": \"%s\", "
           "\"arenas_registered\": %s}\n",
           (int)getpid(), (unsigned long long)o.size, o.chunksize,
           ff->m_files.empty() ? (size_t)0 : ff->m_files.begin()->second->m_chunks.size(), o.batch,
           o.seeder_pipeline ? "true" : "false", o.gpu_encode ? "true" : "false", o.seeder_workers, o.threads,
           serve_s, encode_s, (unsigned long long)sst.requests, (unsigned long long)sst.sent,
           (unsigned long long)sst.refused, sst.verify_s, sst.encode_s, o.corrupt, (unsigned long long)sst.corrupted,
           o.synthetic ? "synthetic stream (generated on request, no seeder file)" : "file",
           o.register_arenas ? "true" : "false");
    fflush(stdout);
    // the leecher has compared its copy before it closed the connection
    if (!o.keep) {
      unlink((seeddir + "/" + name).c_str());
      unlink(floodpath.c_str());
      if (!o.port_file.empty()) unlink(o.port_file.c_str());
      rmdir(seeddir.c_str());
      rmdir(o.dir.c_str());  // whichever peer ends last removes it
    }
    return 0;
  }
  std::thread seeder;
  if (o.role == Opts::BOTH) seeder = std::thread(seeder_main, lfd, ff, seeddir, std::cref(o), std::ref(sst));
  FloodFileSPtr leech_ff(new FloodFile());
  if (leech_ff->FromXMLFile(floodpath) != Error::NO_ERROR_LBF) die("FromXMLFile failed");

  Flood fl;
  fl.m_rootdir = leechdir;
  if (fl.Initialize(leech_ff) != Error::NO_ERROR_LBF) die("leecher: Initialize failed: " + std::string(Encoder::LastError()));
  std::deque<Flood::P_ChunkKey> todo(fl.m_chunkstodownload.begin(), fl.m_chunkstodownload.end());
  const std::vector<Flood::P_ChunkKey> all_keys(todo.begin(), todo.end());
  const size_t total = todo.size();
  // arenas: one filling, one per verifier, one queued for them, one being written
  const int kArenas = (int)o.verifiers + 3;
  const U64 slot = ((U64)o.chunksize + 15) & ~15ull;
  // The arenas live for the whole transfer: pinned once, each batch's verify
  // copies them straight to HBM instead of through the context's staging
  // (lbf_host_register).
  // Registration pins whole pages, so each arena starts on a page of its own.
  const U64 page = (U64)sysconf(_SC_PAGESIZE);
  const U64 arena_len = slot * o.batch, arena_stride = (arena_len + page - 1) / page * page;
  U8* const arena_mem = static_cast<U8*>(aligned_alloc(page, arena_stride * kArenas));
  if (!arena_mem) die("leecher: cannot allocate the arenas");
  memset(arena_mem, 0, arena_stride * kArenas);
  struct Arena {
    U8* p;
    U64 n;
    U8* data() const { return p; }
    U64 size() const { return n; }
  };
  std::vector<Arena> arenas;
  for (int a = 0; a < kArenas; ++a) arenas.push_back(Arena{arena_mem + a * arena_stride, arena_len});
  // --gpu-decode: each arena has a text arena beside it, where the decode
  // stage copies the frames' base64 text (one 16-byte aligned slot per
  // arrival, room for the chunk size's encoded length) for the GPU to decode
  const U64 text_slot = (PeerWire::Base64PutLength(o.chunksize) + 16 + 15) & ~15ull;
  const U64 text_len = o.gpu_decode ? text_slot * o.batch : 0;
  const U64 text_stride = (text_len + page - 1) / page * page;
  U8* const text_mem = o.gpu_decode ? static_cast<U8*>(aligned_alloc(page, text_stride * kArenas)) : nullptr;
  if (o.gpu_decode && !text_mem) die("leecher: cannot allocate the text arenas");
  if (text_mem) memset(text_mem, 0, text_stride * kArenas);
  std::vector<Arena> texts;
  for (int a = 0; a < kArenas && text_mem; ++a) texts.push_back(Arena{text_mem + a * text_stride, text_len});
  // One GPU context per verifier, so their verifies run side by side instead of
  // one after another (a context runs one call at a time), each with a copy of
  // the flood's chunk table (VerifyChunks only reads it).  Verifier 0 uses the
  // process-wide context, like the writer.
  std::vector<lbf_ctx*> vctx(o.verifiers, nullptr);
  vctx[0] = Encoder::Context();
  if (!vctx[0]) die("leecher: no GPU context: " + std::string(Encoder::LastError()));
  for (unsigned v = 1; v < o.verifiers; ++v)
    if (lbf_ctx_create(0, &vctx[v]) != LBF_OK) die(std::string("leecher: lbf_ctx_create: ") + lbf_last_error());
  std::vector<std::unique_ptr<Flood>> vfl;
  for (unsigned v = 0; v < o.verifiers; ++v) {
    vfl.emplace_back(new Flood());
    vfl[v]->m_floodfile = fl.m_floodfile;
    vfl[v]->m_runtimefiles = fl.m_runtimefiles;
    vfl[v]->m_rootdir = fl.m_rootdir;
    vfl[v]->m_ctx = vctx[v];
  }
  if (o.register_arenas)
    for (lbf_ctx* c : vctx)
      for (const std::vector<Arena>* set : {&arenas, &texts})
        for (const Arena& a : *set)
          if (lbf_host_register(c, a.data(), a.size()) != LBF_OK)
            die("leecher: lbf_host_register failed: " + std::string(lbf_last_error()));
  const int fd = connect_loopback(port);

  // Leecher pipeline: reader thread (frames), this thread (decode into one of
  // kArenas arenas, bookkeeping, requests), --verifiers verifier threads
  // (VerifyChunks: the GPU verify, the verdict; each its own context), writer
  // thread (WriteChunks: the accepted chunks to disk, chunkmap '1').
  // ReceiveChunks split in two, so a batch's verify overlaps the next batch's
  // decode and the previous batch's writes, and a slow disk does not hold up
  // verdicts.  With two verifiers a batch never waits for another batch's
  // verify to finish before its own starts.
  struct Batch {
    std::vector<Arrival> got;
    std::vector<Flood::ChunkArrival> arr;
    std::vector<size_t> pos;
    V_U64 text_off;  // --gpu-decode: where each arrival's base64 text lies in its text arena
    V_U32 text_len;
    int arena = 0;
    std::string acc;
    std::string valid;
    Clock::time_point verdict, done;
    double verify_s = 0, write_s = 0;
  };
  Chan<Arrival> arrivals;
  Chan<Batch> to_verify, to_write, verified;
  std::atomic<size_t> in_gpu{0};  // batches handed to the verifier and not yet verified
  std::thread reader([&] {
    FrameReader rd(fd);
    std::string f;
    while (rd.next(f)) arrivals.put(Arrival{std::move(f), Clock::now()});
    arrivals.close();
  });
  std::atomic<unsigned> verifiers_left{o.verifiers};
  std::vector<std::thread> verifier;
  for (unsigned v = 0; v < o.verifiers; ++v)
    verifier.emplace_back([&, v] {
      std::vector<Batch> bs;
      while (to_verify.take(bs, 1)) {
        Batch& b = bs[0];
        auto v0 = Clock::now();
        const Error::ErrorCode rc =
            o.gpu_decode ? vfl[v]->VerifyTextChunks(reinterpret_cast<const char*>(texts[b.arena].data()),
                                                    texts[b.arena].size(), b.text_off, b.text_len, b.arr,
                                                    arenas[b.arena].data(), arenas[b.arena].size(), b.valid)
                         : vfl[v]->VerifyChunks(arenas[b.arena].data(), arenas[b.arena].size(), b.arr, b.valid);
        if (rc != Error::NO_ERROR_LBF) die("leecher: verify failed: " + std::string(Encoder::LastError()));
        b.verdict = Clock::now();
        b.verify_s = secs(v0, b.verdict);
        --in_gpu;
        to_write.put(std::move(b));
      }
      if (--verifiers_left == 0) to_write.close();
    });
  std::thread writer([&] {
    std::vector<Batch> bs;
    while (to_write.take(bs, 1)) {
      Batch& b = bs[0];
      auto w0 = Clock::now();
      if (fl.WriteChunks(arenas[b.arena].data(), b.arr, b.valid, b.acc) != Error::NO_ERROR_LBF)
        die("leecher: WriteChunks failed");
      b.done = Clock::now();
      b.write_s = secs(w0, b.done);
      verified.put(std::move(b));
    }
  });

  std::vector<double> lat_us, acc_us;  // arrival -> verdict, arrival -> written
  lat_us.reserve(total);
  acc_us.reserve(total);
  size_t inflight = 0, accepted = 0, rejected = 0, batches = 0, wire_bytes = 0, undecodable = 0;
  U64 payload = 0;
  double decode_s = 0, verify_s = 0, write_s = 0;
  Flood::S_ChunkKey done;
  std::vector<int> free_arenas;
  for (int a = 0; a < kArenas; ++a) free_arenas.push_back(a);
  const auto t_start = Clock::now();
  auto top_up = [&] {
    if (inflight == 0 && todo.empty() && done.size() < total)  // lost frames: ask again for what is missing
      for (const auto& k : all_keys)
        if (!done.count(k)) todo.push_back(k);
    std::string reqs;
    while (inflight < o.window && !todo.empty()) {
      const Flood::P_ChunkKey k = todo.front();
      todo.pop_front();
      reqs += PeerWire::EncodeMethod(PeerWire::kRequestChunk,
                                     {PeerWire::Value::Str(k.first), PeerWire::Value::Int((int)k.second)});
      ++inflight;
    }
    if (!reqs.empty() && !send_all(fd, reqs)) die("leecher: send failed");
  };
  auto settle = [&](Batch& b) {
    ++batches;
    verify_s += b.verify_s;
    write_s += b.write_s;
    inflight -= b.got.size();
    for (size_t j = 0; j < b.arr.size(); ++j) {
      lat_us.push_back(secs(b.got[b.pos[j]].t, b.verdict) * 1e6);
      acc_us.push_back(secs(b.got[b.pos[j]].t, b.done) * 1e6);
      const Flood::P_ChunkKey key(b.arr[j].m_filename, b.arr[j].m_index);
      if (b.acc[j] == '1') {
        if (done.insert(key).second) {
          ++accepted;
          payload += b.arr[j].m_size;
        }
      } else {
        ++rejected;
        todo.push_front(key);  // ask again
      }
    }
    free_arenas.push_back(b.arena);
    top_up();
  };
  top_up();
  std::vector<Arrival> got;
  std::vector<Batch> res;
  size_t in_verify = 0;
  Pool decode_pool(o.threads);
  while (accepted < total) {
    // settle finished batches first (non-blocking), or wait for one when no arena is free
    {
      std::unique_lock<std::mutex> g(verified.mu);
      if (free_arenas.empty())
        if (!verified.cv.wait_for(g, std::chrono::seconds(120), [&] { return !verified.q.empty(); }))
          die("leecher: verify stalled for 120 s");
      res.clear();
      while (!verified.q.empty()) {
        res.push_back(std::move(verified.q.front()));
        verified.q.pop_front();
      }
    }
    for (Batch& b : res) {
      --in_verify;
      settle(b);
    }
    if (accepted >= total) break;
    if (free_arenas.empty()) continue;
    // next batch of arrivals (wait only if nothing is being verified)
    got.clear();
    {
      std::unique_lock<std::mutex> g(arrivals.mu);
      auto ready = [&] { return !arrivals.q.empty() || arrivals.closed; };
      if (in_verify == 0) {
        if (!arrivals.cv.wait_for(g, std::chrono::seconds(120), ready)) die("leecher: no chunk arrived for 120 s");
      } else {
        // Batches are in flight.  With a verifier idle, start at once.  With
        // every verifier busy, start the next batch once it is full (batches
        // grow to what arrives during one verify) or once its oldest arrival
        // has waited deadline_ms, which bounds the latency that growth adds.
        // With a batch already queued behind them, only a full batch goes: a
        // smaller one would wait for a verifier anyway, and would cost one more
        // chain of verify time.
        const size_t gq = in_gpu.load();
        const auto deadline = std::chrono::milliseconds(o.deadline_ms);
        auto due = [&] {
          if (arrivals.q.size() >= o.batch || arrivals.closed) return true;
          if (arrivals.q.empty()) return false;
          return gq < o.verifiers ||
                 (gq == o.verifiers && o.deadline_ms > 0 && Clock::now() - arrivals.q.front().t >= deadline);
        };
        if (!arrivals.cv.wait_for(g, std::chrono::milliseconds(1), due)) continue;
      }
      while (!arrivals.q.empty() && got.size() < o.batch) {
        got.push_back(std::move(arrivals.q.front()));
        arrivals.q.pop_front();
      }
      if (got.empty() && arrivals.closed && in_verify == 0) die("leecher: seeder closed the connection early");
    }
    if (got.empty()) continue;
    Batch b;
    b.arena = free_arenas.back();
    free_arenas.pop_back();
    U8* arena = arenas[b.arena].data();
    // XmlRpcValue::binaryFromXml + the copy loop of :159-163, on `threads` cores;
    // with --gpu-decode only the frame is parsed here and its base64 text
    // copied to the text arena: the decode runs on the GPU with the verify
    std::vector<Flood::ChunkArrival> arr(got.size());
    std::vector<char> ok(got.size(), 0);
    V_U64 toff(got.size(), 0);
    V_U32 tlen(got.size(), 0);
    U8* const text = o.gpu_decode ? texts[b.arena].data() : nullptr;
    auto d0 = Clock::now();
    decode_pool.run(got.size(), [&](size_t k) {
      size_t n = 0;
      std::string fname;
      U32 idx = 0;
      if (o.gpu_decode) {
        size_t at = 0;
        if (PeerWire::LocateSendChunk(got[k].frame.data(), got[k].frame.size(), fname, idx, at, n) &&
            n <= text_slot) {
          memcpy(text + k * text_slot, got[k].frame.data() + at, n);
          toff[k] = k * text_slot;
          tlen[k] = (U32)n;
          arr[k] = Flood::ChunkArrival{fname, idx, k * slot, 0};
          ok[k] = 1;
        }
      } else if (PeerWire::DecodeSendChunk(got[k].frame.data(), got[k].frame.size(), fname, idx, arena + k * slot,
                                           o.chunksize, n)) {
        arr[k] = Flood::ChunkArrival{fname, idx, k * slot, (U32)n};
        ok[k] = 1;
      }
    });
    decode_s += secs(d0, Clock::now());
    for (size_t k = 0; k < got.size(); ++k) {
      wire_bytes += got[k].frame.size() + 1;
      if (ok[k]) {
        b.arr.push_back(arr[k]);
        b.pos.push_back(k);
        b.text_off.push_back(toff[k]);
        b.text_len.push_back(tlen[k]);
      } else {
        ++undecodable;
      }
    }
    b.got = std::move(got);
    got = std::vector<Arrival>();
    ++in_verify;
    ++in_gpu;
    to_verify.put(std::move(b));
  }
  const auto t_end = Clock::now();
  to_verify.close();
  for (std::thread& t : verifier) t.join();
  writer.join();
  if (o.register_arenas)
    for (lbf_ctx* c : vctx)
      for (const std::vector<Arena>* set : {&arenas, &texts})
        for (const Arena& a : *set) (void)lbf_host_unregister(c, a.data());
  vfl.clear();
  for (unsigned v = 1; v < o.verifiers; ++v) lbf_ctx_destroy(vctx[v]);
  free(arena_mem);
  free(text_mem);

  // end state: what a restarted leecher would find (Flood::_SetupFilesAndChunks),
  // checked while the connection is still open, so a seeder process (which
  // removes its file once the leecher hangs up) still has its copy for the comparison
  Flood check;
  check.m_rootdir = leechdir;
  const bool resumed = check.Initialize(leech_ff) == Error::NO_ERROR_LBF && check.m_chunkstodownload.empty();
  const bool same = o.synthetic ? file_matches_synthetic(leechdir + "/" + name, o.size, o.threads)
                                : files_equal(seeddir + "/" + name, leechdir + "/" + name);
  shutdown(fd, SHUT_RDWR);
  reader.join();
  close(fd);
  if (seeder.joinable()) seeder.join();
  if (lfd >= 0) close(lfd);
  // a leecher process reports the seeder's side as null: the seeder process prints it
  char seeder_json[512];
  if (o.role == Opts::BOTH)
    snprintf(seeder_json, sizeof(seeder_json),
             "{\"requests\": %llu, \"sent\": %llu, \"refused\": %llu, \"verify_s\": %.3f, \"encode_s\": %.3f}",
             (unsigned long long)sst.requests, (unsigned long long)sst.sent, (unsigned long long)sst.refused,
             sst.verify_s, sst.encode_s);
  else
    snprintf(seeder_json, sizeof(seeder_json), "null");
  char corrupted_json[32];
  if (o.role == Opts::BOTH) snprintf(corrupted_json, sizeof(corrupted_json), "%llu", (unsigned long long)sst.corrupted);
  else snprintf(corrupted_json, sizeof(corrupted_json), "null");
  std::sort(lat_us.begin(), lat_us.end());
  std::sort(acc_us.begin(), acc_us.end());
  auto pct_of = [](const std::vector<double>& v, double p) {
    return v.empty() ? 0.0 : v[std::min(v.size() - 1, (size_t)(p * v.size()))];
  };
  auto pct = [&](double p) { return pct_of(lat_us, p); };
  const double wall = secs(t_start, t_end);
  printf("{\"config\": \"C5 loopback 2-peer\", \"role\": \"%s\", \"pid\": %d, \"bytes\": %llu, \"chunk_size\": %u, "
         "\"chunks\": %zu, "
         "\"window\": %u, \"batch\": %u, \"deadline_ms\": %u, \"verifiers\": %u, \"seeder_pipelined\": %s, "
         "\"gpu_decode\": %s, \"gpu_encode\": %s, \"seeder_workers\": %u, "
         "\"threads\": %u, \"seconds\": %.3f, \"payload_gibs\": %.3f, "
         "\"wire_gibs\": %.3f, \"encode_flood_s\": %.3f, "
         "\"leecher\": {\"batches\": %zu, \"mean_batch\": %.1f, \"decode_s\": %.3f, \"verify_s\": %.3f, "
         "\"write_s\": %.3f, "
         "\"rejected\": %zu, \"undecodable\": %zu}, \"seeder\": %s, "
         "\"verify_latency_us\": {\"p50\": %.0f, \"p90\": %.0f, \"p99\": %.0f, \"max\": %.0f}, "
         "\"accept_latency_us\": {\"p50\": %.0f, \"p90\": %.0f, \"p99\": %.0f, \"max\": %.0f}, "
         "\"resume_verify_complete\": %s, \"files_identical\": %s, \"corrupt_every\": %u, \"corrupted_sent\": %s, "
         "\"seed_source\": \"%s\", \"arenas_registered\": %s}\n",
         o.role == Opts::BOTH ? "both" : "leecher", (int)getpid(), (unsigned long long)o.size, o.chunksize, total,
         o.window, o.batch, o.deadline_ms, o.verifiers,
         o.seeder_pipeline ? "true" : "false", o.gpu_decode ? "true" : "false",
         o.gpu_encode ? "true" : "false", o.seeder_workers, o.threads, wall,
         payload / wall / (1u << 30), wire_bytes / wall / (1u << 30), encode_s, batches,
         batches ? (double)(accepted + rejected) / batches : 0.0, decode_s, verify_s, write_s, rejected, undecodable,
         seeder_json, pct(0.5), pct(0.9), pct(0.99), lat_us.empty() ? 0.0 : lat_us.back(), pct_of(acc_us, 0.5),
         pct_of(acc_us, 0.9), pct_of(acc_us, 0.99), acc_us.empty() ? 0.0 : acc_us.back(), resumed ? "true" : "false",
         same ? "true" : "false", o.corrupt, corrupted_json,
         o.synthetic ? "synthetic stream (generated on request, no seeder file)" : "file",
         o.register_arenas ? "true" : "false");
  if (!o.keep) {
    unlink((leechdir + "/" + name).c_str());
    rmdir(leechdir.c_str());
    if (o.role == Opts::BOTH) {  // a seeder process removes its own files
      unlink((seeddir + "/" + name).c_str());
      unlink(floodpath.c_str());
      rmdir(seeddir.c_str());
    }
    rmdir(o.dir.c_str());
  }
  return resumed && same ? 0 : 1;
}
