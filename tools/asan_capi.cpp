// tools/asan_capi.cpp -- diagnostic (not product code): randomized stress of the
// C ABI's host paths (include/lbf_hash.h) in a build whose HOST code carries
// AddressSanitizer + UBSan (tools/asan_build.sh; device code is not
// instrumented).  Each case draws a context shape (workers per device,
// staging slots, slot size, an injected one-shot group fault) and a batch
// (ragged, unaligned, empty and oversize chunks), then checks
//   lbf_sha1_batch / lbf_verify_batch (host memory) and
//   lbf_file_ranges (hash and verify, including a truncated file) and
//   lbf_files_ranges (verify over 2-4 truncated or missing files)
//   lbf_verify_encode_b64_batch + lbf_b64_verify_batch (the wire form both ways:
//   text slots at ragged offsets, some texts cut short; no byte between slots
//   written, a short decode's slot tail zeroed)
// with pageable jobs pinned on the fly in half of the contexts (LBF_AUTOPIN*),
// against the oracle (oracle/sha1_oracle.c, compiled in as the checker).  Half
// the jobs read from memory registered with the context, and half the
// contexts then take three concurrent callers with 24-40 MiB batches (enough
// for the staging-copy helper threads), so a ThreadSanitizer build of the
// same driver (tools/tsan_build.sh) sees every host thread the pipeline runs.
//   asan_capi <scratch-dir> [seconds] [seed]
#include <fcntl.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "lbf_hash.h"

extern "C" {
void oracle_sha1(const uint8_t* data, uint32_t len, uint8_t out[20]);
void oracle_synth_fill_mt(uint8_t* out, uint64_t len, uint64_t seed, uint64_t start, int nthreads);
}

static std::atomic<int> g_fail{0};
#define CHECK(cond, ...)                                                  \
  do {                                                                    \
    if (!(cond)) {                                                        \
      std::fprintf(stderr, "CHECK failed %s:%d: %s: ", __FILE__, __LINE__, #cond); \
      std::fprintf(stderr, __VA_ARGS__);                                  \
      std::fprintf(stderr, "\n");                                         \
      ++g_fail;                                                           \
    }                                                                     \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: asan_capi <scratch-dir> [seconds] [seed]\n");
    return 2;
  }
  const std::string dir = argv[1];
  const double budget = argc > 2 ? atof(argv[2]) : 60.0;
  const uint64_t seed = argc > 3 ? strtoull(argv[3], nullptr, 10) : 1;
  std::mt19937_64 rng(seed);
  auto uni = [&](uint64_t lo, uint64_t hi) { return lo + rng() % (hi - lo + 1); };
  const auto t_end = std::chrono::steady_clock::now() + std::chrono::duration<double>(budget);
  long cases = 0, chunks_checked = 0, faults = 0, registered = 0, concurrent = 0;
  const std::string path = dir + "/asan_capi.bin";

  while (std::chrono::steady_clock::now() < t_end && g_fail.load() == 0) {
    // ---- context shape (environment read at creation) ----
    const int workers = (int)uni(1, 4), slots = (int)uni(2, 5), slot_mb = (int)(uni(0, 3) == 0 ? 1 : uni(2, 16));
    const bool fault = uni(0, 4) == 0;
    setenv("LBF_WORKERS_PER_DEVICE", std::to_string(workers).c_str(), 1);
    setenv("LBF_SLOTS", std::to_string(slots).c_str(), 1);
    setenv("LBF_SLOT_MB", std::to_string(slot_mb).c_str(), 1);
    setenv("LBF_TEST_FAULT_GROUP", fault ? std::to_string(uni(0, 3)).c_str() : "-1", 1);
    setenv("LBF_TEST_FAULT_WORKER", std::to_string(uni(0, workers - 1)).c_str(), 1);
    // on-the-fly pinning of pageable jobs (read per job): off or on, from 1 MiB of job on
    setenv("LBF_AUTOPIN", uni(0, 1) ? "1" : "0", 1);
    setenv("LBF_AUTOPIN_MIN_MB", "1", 1);
    lbf_ctx* ctx = nullptr;
    if (lbf_ctx_create(1, &ctx) != LBF_OK) {
      std::fprintf(stderr, "lbf_ctx_create: %s\n", lbf_last_error());
      return 2;
    }
    for (int job = 0; job < 3; ++job) {
      // ---- batch ----
      const uint64_t buf_len = uni(1, 12) << 20;
      std::vector<uint8_t> buf(buf_len);
      oracle_synth_fill_mt(buf.data(), buf_len, rng(), 0, 4);
      // a quarter of the tables cover a span of the buffer without a gap (from a
      // random start byte, any chunk size): the shape on-the-fly pinning takes,
      // its inward page rounding and the bounce of the partial edge pages
      const bool tiled = uni(0, 3) == 0;
      const uint64_t t_lo = tiled ? uni(0, buf_len / 4) : 0, t_cs = tiled ? uni(1, 600000) : 1;
      const uint64_t n = tiled ? (buf_len - t_lo + t_cs - 1) / t_cs : uni(0, 1) ? uni(0, 40) : uni(0, 1500);
      std::vector<uint64_t> off(n);
      std::vector<uint32_t> size(n);
      for (uint64_t i = 0; i < n; ++i) {
        if (tiled) {
          off[i] = t_lo + i * t_cs;
          size[i] = (uint32_t)std::min<uint64_t>(t_cs, buf_len - off[i]);
          continue;
        }
        const int kind = (int)uni(0, 9);
        uint64_t s = kind == 0 ? uni(0, 130) : kind == 1 ? uni(1, 3) << 20 : uni(0, kind < 5 ? 70000 : 300000);
        s = std::min<uint64_t>(s, buf_len);
        size[i] = (uint32_t)s;
        off[i] = uni(0, buf_len - s);
        if (uni(0, 2) == 0) off[i] &= ~63ull;
      }
      std::vector<uint8_t> want(20 * n), got(20 * n, 0xEE);
      for (uint64_t i = 0; i < n; ++i) oracle_sha1(buf.data() + off[i], size[i], &want[20 * i]);
      ++cases;
      // half the jobs read from memory registered with the context (the direct route)
      const bool reg = uni(0, 1) == 0;
      if (reg) CHECK(lbf_host_register(ctx, buf.data(), buf_len) == LBF_OK, "register: %s", lbf_last_error());
      registered += reg;
      int rc = lbf_sha1_batch(ctx, buf.data(), buf_len, off.data(), size.data(), n, got.data(), LBF_HOST_PTR);
      if (rc == LBF_ERR_HIP && strstr(lbf_last_error(), "injected fault")) {
        ++faults;  // one-shot: the same job must now succeed on the same context
        rc = lbf_sha1_batch(ctx, buf.data(), buf_len, off.data(), size.data(), n, got.data(), LBF_HOST_PTR);
      }
      CHECK(rc == LBF_OK, "hash rc %d: %s", rc, lbf_last_error());
      for (uint64_t i = 0; i < n && rc == LBF_OK; ++i)
        CHECK(memcmp(&got[20 * i], &want[20 * i], 20) == 0, "hash chunk %lu size %u off %lu", (unsigned long)i,
              size[i], (unsigned long)off[i]);
      chunks_checked += (long)n;
      // verify with some expected digests corrupted
      std::vector<uint8_t> exp = want, ver(n, 7);
      std::vector<uint8_t> bad(n, 0);
      for (uint64_t i = 0; i < n; ++i)
        if (uni(0, 7) == 0) {
          exp[20 * i + uni(0, 19)] ^= (uint8_t)(1u << uni(0, 7));
          bad[i] = 1;
        }
      rc = lbf_verify_batch(ctx, buf.data(), buf_len, off.data(), size.data(), n, exp.data(), ver.data(), LBF_HOST_PTR);
      if (rc == LBF_ERR_HIP && strstr(lbf_last_error(), "injected fault")) {
        ++faults;
        rc = lbf_verify_batch(ctx, buf.data(), buf_len, off.data(), size.data(), n, exp.data(), ver.data(),
                              LBF_HOST_PTR);
      }
      CHECK(rc == LBF_OK, "verify rc %d: %s", rc, lbf_last_error());
      for (uint64_t i = 0; i < n && rc == LBF_OK; ++i) CHECK(ver[i] == (bad[i] ? 0 : 1), "verdict %lu", (unsigned long)i);
      if (reg) CHECK(lbf_host_unregister(ctx, buf.data()) == LBF_OK, "unregister: %s", lbf_last_error());
      // the same chunks from a file, truncated in half of the cases
      const uint64_t keep = uni(0, 1) ? buf_len : uni(0, buf_len);
      const int fd = open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
      CHECK(fd >= 0 && write(fd, buf.data(), keep) == (ssize_t)keep, "write %s", path.c_str());
      close(fd);
      std::vector<uint8_t> fver(n, 7);
      rc = lbf_file_ranges(ctx, path.c_str(), off.data(), size.data(), n, want.data(), fver.data());
      if (rc == LBF_ERR_HIP && strstr(lbf_last_error(), "injected fault")) {
        ++faults;
        rc = lbf_file_ranges(ctx, path.c_str(), off.data(), size.data(), n, want.data(), fver.data());
      }
      CHECK(rc == LBF_OK, "file verify rc %d: %s", rc, lbf_last_error());
      bool all_present = true;
      for (uint64_t i = 0; i < n && rc == LBF_OK; ++i) {
        const bool present = size[i] == 0 || off[i] + size[i] <= keep;
        all_present = all_present && present;
        CHECK(fver[i] == (present ? 1 : 0), "file verdict %lu", (unsigned long)i);
      }
      std::vector<uint8_t> fdig(20 * n, 0);
      rc = lbf_file_ranges(ctx, path.c_str(), off.data(), size.data(), n, nullptr, fdig.data());
      if (rc == LBF_ERR_HIP && strstr(lbf_last_error(), "injected fault")) {
        ++faults;
        rc = lbf_file_ranges(ctx, path.c_str(), off.data(), size.data(), n, nullptr, fdig.data());
      }
      if (all_present) {
        CHECK(rc == LBF_OK, "file hash rc %d: %s", rc, lbf_last_error());
        CHECK(n == 0 || memcmp(fdig.data(), want.data(), 20 * n) == 0, "file digests");
      } else {
        CHECK(rc == LBF_ERR_IO, "file hash of a truncated file rc %d: %s", rc, lbf_last_error());
      }
      // several files at once (lbf_files_ranges): the buffer's bytes spread over
      // 2-4 files that each hold a copy truncated at its own length, one maybe
      // missing; every chunk names a random file
      const uint32_t nf = (uint32_t)uni(2, 4);
      std::vector<std::string> fpaths(nf);
      std::vector<uint64_t> fkeep(nf);
      std::vector<bool> fmissing(nf, false);
      for (uint32_t f = 0; f < nf; ++f) {
        fpaths[f] = dir + "/asan_capi_f" + std::to_string(f) + ".bin";
        fmissing[f] = uni(0, 5) == 0;
        fkeep[f] = uni(0, 2) ? buf_len : uni(0, buf_len);
        unlink(fpaths[f].c_str());
        if (fmissing[f]) continue;
        const int g = open(fpaths[f].c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
        CHECK(g >= 0 && write(g, buf.data(), fkeep[f]) == (ssize_t)fkeep[f], "write %s", fpaths[f].c_str());
        close(g);
      }
      std::vector<const char*> cp(nf);
      for (uint32_t f = 0; f < nf; ++f) cp[f] = fpaths[f].c_str();
      std::vector<uint32_t> file_of(n);
      for (uint64_t i = 0; i < n; ++i) file_of[i] = (uint32_t)uni(0, nf - 1);
      std::vector<uint8_t> mver(n, 7);
      rc = lbf_files_ranges(ctx, cp.data(), nf, file_of.data(), off.data(), size.data(), n, want.data(), mver.data());
      if (rc == LBF_ERR_HIP && strstr(lbf_last_error(), "injected fault")) {
        ++faults;
        rc = lbf_files_ranges(ctx, cp.data(), nf, file_of.data(), off.data(), size.data(), n, want.data(), mver.data());
      }
      CHECK(rc == LBF_OK, "files verify rc %d: %s", rc, lbf_last_error());
      for (uint64_t i = 0; i < n && rc == LBF_OK; ++i) {
        const uint32_t f = file_of[i];
        const bool present = !fmissing[f] && (size[i] == 0 || off[i] + size[i] <= fkeep[f]);
        CHECK(mver[i] == (present ? 1 : 0), "files verdict %lu (file %u)", (unsigned long)i, f);
      }
      for (uint32_t f = 0; f < nf; ++f) unlink(fpaths[f].c_str());
      // the wire form both ways: encode (with the corrupted digests above) into
      // text slots at ragged offsets between sentinels, then decode the texts
      // back, some cut short, against the true digests
      {
        const uint64_t m = std::min<uint64_t>(n, 200);
        std::vector<uint64_t> toff(m), ooff(m);
        std::vector<uint32_t> tlen(m), dlen(m), dsz(m, 0);
        uint64_t tpos = uni(0, 40), opos = uni(0, 40);
        for (uint64_t i = 0; i < m; ++i) {
          toff[i] = tpos;
          tlen[i] = (uint32_t)lbf_b64_put_length(size[i]);
          tpos += tlen[i] + uni(0, 40);
          ooff[i] = opos;
          opos += size[i] + uni(0, 40);
        }
        const uint64_t thead = m ? toff[0] : 0, ohead = m ? ooff[0] : 0;
        const uint64_t ttail = m ? toff[m - 1] + tlen[m - 1] : 0, otail = m ? ooff[m - 1] + size[m - 1] : 0;
        std::vector<char> text(tpos + 64, '\x01');
        std::vector<uint8_t> ev(m, 7), dv(m, 7), cut(m, 0), out(opos + 64, 0xA5);
        rc = lbf_verify_encode_b64_batch(ctx, buf.data(), buf_len, off.data(), size.data(), m, exp.data(), ev.data(),
                                         text.data(), text.size(), toff.data());
        CHECK(rc == LBF_OK, "encode rc %d: %s", rc, lbf_last_error());
        for (uint64_t i = 0; i < m && rc == LBF_OK; ++i) CHECK(ev[i] == (bad[i] ? 0 : 1), "encode verdict %lu", (unsigned long)i);
        for (uint64_t k = 0; k < thead; ++k) CHECK(text[k] == '\x01', "text byte %lu before the first slot", (unsigned long)k);
        for (uint64_t k = ttail; k < text.size(); ++k) CHECK(text[k] == '\x01', "text byte %lu after the last slot", (unsigned long)k);
        for (uint64_t i = 0; i + 1 < m; ++i)  // between slots too: results come back slot by slot
          for (uint64_t k = toff[i] + tlen[i]; k < toff[i + 1]; ++k)
            CHECK(text[k] == '\x01', "text byte %lu between slots %lu and %lu", (unsigned long)k, (unsigned long)i,
                  (unsigned long)i + 1);
        for (uint64_t i = 0; i < m; ++i) {
          dlen[i] = tlen[i];
          if (tlen[i] >= 8 && uni(0, 5) == 0) {  // lose at least one group
            dlen[i] = (uint32_t)uni(0, tlen[i] - 4);
            cut[i] = 1;
          }
        }
        rc = lbf_b64_verify_batch(ctx, text.data(), text.size(), toff.data(), dlen.data(), m, size.data(), want.data(),
                                  out.data(), out.size(), ooff.data(), dsz.data(), dv.data());
        CHECK(rc == LBF_OK, "decode rc %d: %s", rc, lbf_last_error());
        for (uint64_t i = 0; i < m && rc == LBF_OK; ++i) {
          CHECK(dv[i] == (cut[i] ? 0 : 1), "decode verdict %lu (cut %d)", (unsigned long)i, cut[i]);
          CHECK(cut[i] ? dsz[i] < size[i] : dsz[i] == size[i], "decoded size %lu: %u of %u", (unsigned long)i, dsz[i],
                size[i]);
          if (!cut[i])
            CHECK(memcmp(out.data() + ooff[i], buf.data() + off[i], size[i]) == 0, "decoded bytes %lu", (unsigned long)i);
          else  // a short decode leaves zeros in the rest of its slot, never stale device bytes
            for (uint64_t k = dsz[i]; k < size[i]; ++k)
              CHECK(out[ooff[i] + k] == 0, "slot %lu byte %lu past a short decode", (unsigned long)i, (unsigned long)k);
        }
        for (uint64_t i = 0; i + 1 < m; ++i)
          for (uint64_t k = ooff[i] + size[i]; k < ooff[i + 1]; ++k)
            CHECK(out[k] == 0xA5, "out byte %lu between slots %lu and %lu", (unsigned long)k, (unsigned long)i,
                  (unsigned long)i + 1);
        for (uint64_t k = 0; k < ohead; ++k) CHECK(out[k] == 0xA5, "out byte %lu before the first slot", (unsigned long)k);
        for (uint64_t k = otail; k < out.size(); ++k) CHECK(out[k] == 0xA5, "out byte %lu after the last slot", (unsigned long)k);
        chunks_checked += (long)(2 * m);
      }
    }
    if (uni(0, 1) == 0) {
      // three concurrent callers on this context (calls serialize on its
      // mutex; each runs the multi-worker split and the copy helpers inside)
      std::vector<uint64_t> seeds(3);
      for (uint64_t& x : seeds) x = rng();
      std::atomic<long> done_chunks{0}, done_faults{0};
      std::vector<std::thread> callers;
      for (int t = 0; t < 3; ++t)
        callers.emplace_back([&, t] {
          std::mt19937_64 r(seeds[t]);
          auto u = [&](uint64_t lo, uint64_t hi) { return lo + r() % (hi - lo + 1); };
          const uint64_t len = u(24, 40) << 20;
          std::vector<uint8_t> b(len);
          oracle_synth_fill_mt(b.data(), len, r(), 0, 2);
          const uint64_t cs = u(0, 1) ? 262144 : u(1, 3) << 20;
          const uint64_t n = (len + cs - 1) / cs;
          std::vector<uint64_t> o(n);
          std::vector<uint32_t> z(n);
          for (uint64_t i = 0; i < n; ++i) o[i] = i * cs, z[i] = (uint32_t)std::min<uint64_t>(cs, len - i * cs);
          std::vector<uint8_t> w(20 * n), g(20 * n, 0xEE);
          for (uint64_t i = 0; i < n; ++i) oracle_sha1(b.data() + o[i], z[i], &w[20 * i]);
          const bool rg = u(0, 1) == 0;
          if (rg) CHECK(lbf_host_register(ctx, b.data(), len) == LBF_OK, "register: %s", lbf_last_error());
          int rc = lbf_sha1_batch(ctx, b.data(), len, o.data(), z.data(), n, g.data(), LBF_HOST_PTR);
          if (rc == LBF_ERR_HIP && strstr(lbf_last_error(), "injected fault")) {
            ++done_faults;
            rc = lbf_sha1_batch(ctx, b.data(), len, o.data(), z.data(), n, g.data(), LBF_HOST_PTR);
          }
          CHECK(rc == LBF_OK, "concurrent hash rc %d: %s", rc, lbf_last_error());
          CHECK(rc != LBF_OK || memcmp(g.data(), w.data(), 20 * n) == 0, "concurrent digests (caller %d)", t);
          if (rg) CHECK(lbf_host_unregister(ctx, b.data()) == LBF_OK, "unregister: %s", lbf_last_error());
          done_chunks += (long)n;
        });
      for (auto& c : callers) c.join();
      chunks_checked += done_chunks.load();
      faults += done_faults.load();
      cases += 3;
      concurrent += 3;
    }
    if (uni(0, 2) == 0) {
      // two contexts: a job pinned on the fly (LBF_AUTOPIN=1, read per job)
      // while another context registers a range inside its pages, and a third
      // thread pins the page the job shares with its neighbour (round 6: the
      // job's pages are never adopted, the edge page is never the job's)
      setenv("LBF_AUTOPIN", "1", 1);
      setenv("LBF_TEST_FAULT_GROUP", "-1", 1);  // read at creation: the second context injects nothing
      lbf_ctx* other = nullptr;
      CHECK(lbf_ctx_create(1, &other) == LBF_OK, "second context: %s", lbf_last_error());
      const uint64_t page = (uint64_t)sysconf(_SC_PAGESIZE), len = uni(8, 24) << 20;
      std::vector<uint8_t> b(len + 2 * page);
      const uint64_t skew = uni(1, page - 1);  // the job starts and ends inside shared pages
      uint8_t* job = b.data() + skew;
      const uint64_t jlen = len;
      oracle_synth_fill_mt(job, jlen, rng(), 0, 2);
      const uint64_t cs = uni(1, 3) << 18, n = (jlen + cs - 1) / cs;
      std::vector<uint64_t> o(n);
      std::vector<uint32_t> z(n);
      for (uint64_t i = 0; i < n; ++i) o[i] = i * cs, z[i] = (uint32_t)std::min<uint64_t>(cs, jlen - i * cs);
      std::vector<uint8_t> w(20 * n), g(20 * n, 0xEE);
      for (uint64_t i = 0; i < n; ++i) oracle_sha1(job + o[i], z[i], &w[20 * i]);
      const uint64_t sub_lo = ((uint64_t)(job - b.data()) + jlen / 4 + page - 1) / page * page;
      uint8_t* sub = b.data() + sub_lo;
      const uint64_t sub_len = jlen / 4;
      std::thread a([&] {
        const int rc = lbf_sha1_batch(ctx, job, jlen, o.data(), z.data(), n, g.data(), LBF_HOST_PTR);
        CHECK(rc == LBF_OK || strstr(lbf_last_error(), "injected fault"), "pinned-on-the-fly job rc %d: %s", rc,
              lbf_last_error());
        CHECK(rc != LBF_OK || memcmp(g.data(), w.data(), 20 * n) == 0, "pinned-on-the-fly job digests");
      });
      std::thread r([&] {
        CHECK(lbf_host_register(other, sub, sub_len) == LBF_OK, "register beside a job: %s", lbf_last_error());
        std::vector<uint64_t> so{0};
        std::vector<uint32_t> ss{(uint32_t)sub_len};
        std::vector<uint8_t> sd(20), sw(20);
        oracle_sha1(sub, sub_len, sw.data());
        CHECK(lbf_sha1_batch(other, sub, sub_len, so.data(), ss.data(), 1, sd.data(), LBF_HOST_PTR) == LBF_OK,
              "hash of the registered sub-range: %s", lbf_last_error());
        CHECK(memcmp(sd.data(), sw.data(), 20) == 0, "registered sub-range digest");
        CHECK(lbf_host_unregister(other, sub) == LBF_OK, "unregister: %s", lbf_last_error());
      });
      a.join();
      r.join();
      lbf_ctx_destroy(other);
      cases += 2;
      concurrent += 2;
      chunks_checked += (long)n + 1;
    }
    lbf_ctx_destroy(ctx);
  }
  unlink(path.c_str());
  std::printf("asan_capi %s: %ld cases (%ld from registered memory, %ld concurrent callers), %ld chunks, "
              "%ld injected faults, seed %lu\n",
              g_fail ? "FAIL" : "OK", cases, registered, concurrent, chunks_checked, faults, (unsigned long)seed);
  std::fflush(stdout);
  // Skip static destructors: the HIP runtime's own teardown (libamdhip64
  // __cxa_finalize) can trip ASan's device-allocator CHECK
  // (sanitizer_allocator_device.h "dev_runtime_unloaded_") after ROCr has
  // unloaded -- a runtime/ASan interaction at exit, not a finding in this code.
  _exit(g_fail ? 1 : 0);
}
