// gpu_tests.cpp -- C++ API tests that need the GPU (run by
// tests/test_host_cpp.py under -m gpu): Base64Encode KATs through the
// reference signature, the batch extension, and the seeder/receiver verify
// paths of Flood (ChunkMethods.cpp:89-225 restated) on a real file.
//   lbf_gpu_tests <scratch-dir>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "libBitFlood/Encoder.H"
#include "libBitFlood/Flood.H"
#include "libBitFlood/PeerWire.H"

using namespace libBitFlood;

static int g_fail = 0;
#define CHECK(cond)                                                                  \
  do {                                                                               \
    if (!(cond)) {                                                                   \
      std::fprintf(stderr, "%s:%d CHECK failed: %s\n", __FILE__, __LINE__, #cond);   \
      ++g_fail;                                                                      \
    }                                                                                \
  } while (0)

static std::vector<U8> pattern(size_t n, U32 seed) {
  std::vector<U8> v(n);
  U32 x = seed * 2654435761u + 1;
  for (size_t i = 0; i < n; ++i) {
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    v[i] = (U8)(x >> 24);
  }
  return v;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: lbf_gpu_tests <scratch-dir>\n");
    return 2;
  }
  const std::string dir = argv[1];
  FloodFile::SetResolveTrackerHosts(false);

  // Base64Encode through the reference signature (sha.txt KATs, Encoder.cpp:107-120)
  std::string s;
  if (Encoder::Base64Encode((const U8*)"abc", 3, s) != Error::NO_ERROR_LBF) {
    std::fprintf(stderr, "no GPU path: %s\n", Encoder::LastError());
    return 1;
  }
  CHECK(s == "qZk+NkcGgWq6PiVxeFDCbJzQ2J0");
  CHECK(Encoder::Base64Encode((const U8*)"", 0, s) == Error::NO_ERROR_LBF);
  CHECK(s == "2jmj7l5rSw0yVb/vlWAYkK/YBwk");
  const char* nist = "abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq";
  Encoder::Base64Encode((const U8*)nist, (U32)strlen(nist), s);
  CHECK(s == "hJg+RBw70m66rkqh+VEp5eVGcPE");

  // batch == per-buffer
  std::vector<U8> buf = pattern(1 << 20, 3);
  std::vector<U64> offs = {0, 1, 64, 4096, 100000};
  std::vector<U32> sizes = {0, 55, 56, 65536, 300000};
  V_String hs;
  CHECK(Encoder::Base64EncodeBatch(buf.data(), buf.size(), offs.data(), sizes.data(), offs.size(), hs) ==
        Error::NO_ERROR_LBF);
  for (size_t i = 0; i < offs.size() && i < hs.size(); ++i) {
    std::string one;
    Encoder::Base64Encode(buf.data() + offs[i], sizes[i], one);
    CHECK(hs[i] == one);
  }

  // Base64Encode from several threads at once, as the reference's reentrant
  // call allows (a stack hasher per call, Encoder.cpp:107-120): each thread's
  // strings equal the ones computed one call at a time above
  {
    std::vector<std::string> one(64);
    std::vector<U32> at(64), len(64);
    for (U32 k = 0; k < 64; ++k) {
      at[k] = (k * 7919u) % 500000u;
      len[k] = (k * 104729u) % 300000u;
      Encoder::Base64Encode(buf.data() + at[k], len[k], one[k]);
    }
    std::vector<int> bad(8, 0);
    std::vector<std::thread> th;
    for (int t = 0; t < 8; ++t)
      th.emplace_back([&, t] {
        for (int rep = 0; rep < 3; ++rep)
          for (U32 k = (U32)t; k < 64; k += 2) {
            std::string s2;
            if (Encoder::Base64Encode(buf.data() + at[k], len[k], s2) != Error::NO_ERROR_LBF || s2 != one[k]) ++bad[t];
          }
        V_String many;
        std::vector<U64> o(at.begin(), at.end());
        if (Encoder::Base64EncodeBatch(buf.data(), buf.size(), o.data(), len.data(), 64, many) != Error::NO_ERROR_LBF ||
            many != one)
          ++bad[t];
      });
    for (auto& x : th) x.join();
    for (int t = 0; t < 8; ++t) CHECK(bad[t] == 0);

    // SetDeviceMask replaces the process context while other threads hash:
    // their calls keep the context they started with (shared ownership), so
    // every result is still exact and nothing runs on a destroyed context.
    std::atomic<bool> stop{false};
    std::vector<int> bad2(4, 0);
    std::vector<std::thread> th2;
    for (int t = 0; t < 4; ++t)
      th2.emplace_back([&, t] {
        for (U32 k = (U32)t; !stop; k = (k + 4) % 64) {
          std::string s2;
          if (Encoder::Base64Encode(buf.data() + at[k], len[k], s2) != Error::NO_ERROR_LBF || s2 != one[k]) ++bad2[t];
        }
      });
    for (int sw = 0; sw < 20; ++sw) {
      CHECK(Encoder::SetDeviceMask(sw & 1 ? 1u : 0u) == Error::NO_ERROR_LBF);
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
    stop = true;
    for (auto& x : th2) x.join();
    for (int t = 0; t < 4; ++t) CHECK(bad2[t] == 0);
    CHECK(Encoder::SetDeviceMask(0) == Error::NO_ERROR_LBF);
  }

  // EncodeFile -> Flood: seeder read-verify, receiver accept/reject
  const std::string src = dir + "/seed.bin";
  std::vector<U8> data = pattern(3 * 65536 + 777, 9);
  FILE* f = std::fopen(src.c_str(), "wb");
  std::fwrite(data.data(), 1, data.size(), f);
  std::fclose(f);
  Encoder::ToEncode e;
  e.m_files.push_back(src);
  e.m_chunksize = 65536;
  e.m_trackers.push_back({"127.0.0.1", 10101});
  FloodFileSPtr ff(new FloodFile());
  CHECK(Encoder::EncodeFile(e, *ff) == Error::NO_ERROR_LBF);
  CHECK(ff->m_files.size() == 1 && ff->m_files[src]->m_chunks.size() == 4);
  CHECK(ff->m_files[src]->m_size == data.size());

  Flood seeder;
  CHECK(seeder.Initialize(ff) == Error::NO_ERROR_LBF);
  CHECK(seeder.m_runtimefiles[src].m_chunkmap == "1111");
  CHECK(seeder.m_chunkstodownload.empty());
  V_U8 chunk;
  bool valid = false;
  CHECK(seeder.ReadVerifiedChunk(src, 3, chunk, valid) == Error::NO_ERROR_LBF);
  CHECK(valid && chunk.size() == 777 && std::memcmp(chunk.data(), data.data() + 3 * 65536, 777) == 0);

  // a leecher whose copy lives elsewhere: same flood, empty directory
  const std::string ldir = dir + "/leech";
  std::string mk = "mkdir -p '" + ldir + "'";
  CHECK(std::system(mk.c_str()) == 0);
  FloodFileSPtr lf(new FloodFile());
  FloodFile::FileSPtr lfile(new FloodFile::File(*ff->m_files[src]));
  lfile->m_name = "copy.bin";
  lf->m_files["copy.bin"] = lfile;
  Flood leech;
  leech.m_rootdir = ldir;
  CHECK(leech.Initialize(lf) == Error::NO_ERROR_LBF);
  CHECK(leech.m_runtimefiles["copy.bin"].m_chunkmap == "0000");
  CHECK(leech.m_chunkstodownload.size() == 4);
  bool accepted = true;
  std::vector<U8> bad(data.begin() + 65536, data.begin() + 2 * 65536);
  bad[17] ^= 1;
  CHECK(leech.ReceiveChunk("copy.bin", 1, bad.data(), (U32)bad.size(), accepted) == Error::NO_ERROR_LBF);
  CHECK(!accepted);  // corrupted: dropped (ChunkMethods.cpp:167)
  CHECK(leech.ReceiveChunk("copy.bin", 1, data.data() + 65536, 1000, accepted) == Error::NO_ERROR_LBF);
  CHECK(!accepted);  // wrong size (ChunkMethods.cpp:156)
  for (U32 i : {3u, 1u, 0u, 2u}) {  // out of order, like a swarm
    const U32 sz = i == 3 ? 777 : 65536;
    CHECK(leech.ReceiveChunk("copy.bin", i, data.data() + 65536ull * i, sz, accepted) == Error::NO_ERROR_LBF);
    CHECK(accepted);
  }
  CHECK(leech.m_runtimefiles["copy.bin"].m_chunkmap == "1111");
  CHECK(leech.m_chunkstodownload.empty());
  // the written file re-verifies from scratch (resume after restart)
  Flood again;
  again.m_rootdir = ldir;
  CHECK(again.Initialize(lf) == Error::NO_ERROR_LBF);
  CHECK(again.m_runtimefiles["copy.bin"].m_chunkmap == "1111");

  // the wire form end to end: the seeder's verify + encode on the GPU
  // (VerifyEncodeChunks) frames the same bytes as EncodeSendChunk; a receiver
  // decoding those frames on the GPU (VerifyTextChunks) accepts every chunk
  // but the one whose expected size disagrees and the one flipped on the wire
  {
    std::vector<Flood::ChunkArrival> out(5);
    V_U64 toff(5);
    for (U32 i = 0; i < 4; ++i) {
      out[i] = Flood::ChunkArrival{src, i, 65536ull * i, i == 3 ? 777u : 65536u};
      toff[i] = 90000ull * i;
    }
    out[4] = Flood::ChunkArrival{src, 2, 65536ull * 2, 1000};  // wrong size: skipped
    toff[4] = 90000ull * 4;
    std::vector<char> text(90000 * 5, 0);
    std::string ok;
    CHECK(seeder.VerifyEncodeChunks(data.data(), data.size(), out, ok, text.data(), text.size(), toff) ==
          Error::NO_ERROR_LBF);
    CHECK(ok == "11110");
    std::vector<std::string> frames;
    for (U32 i = 0; i < 4; ++i) {
      const U32 sz = out[i].m_size;
      frames.push_back(PeerWire::FrameSendChunkText(src, i, &text[toff[i]], PeerWire::Base64PutLength(sz)));
      CHECK(frames.back() == PeerWire::EncodeSendChunk(src, i, data.data() + 65536ull * i, sz));
    }
    std::string& f1 = frames[1];  // a character flipped in transit
    const size_t at = f1.find("<base64>") + 8 + 100;
    f1[at] = f1[at] == 'A' ? 'B' : 'A';
    std::string all;
    V_U64 boff;
    V_U32 blen;
    std::vector<Flood::ChunkArrival> got;
    for (U32 i = 0; i < 4; ++i) {
      std::string fname;
      U32 idx = 0;
      size_t b = 0, n = 0;
      CHECK(PeerWire::LocateSendChunk(frames[i].data(), frames[i].size(), fname, idx, b, n) && idx == i);
      boff.push_back(all.size() + b);
      blen.push_back((U32)n);
      got.push_back(Flood::ChunkArrival{"copy.bin", idx, 65536ull * i, 0});
      all += frames[i];
    }
    Flood leech2;
    leech2.m_rootdir = ldir;
    CHECK(leech2.Initialize(lf) == Error::NO_ERROR_LBF);
    std::vector<U8> arena(4 * 65536);
    std::string valid;
    CHECK(leech2.VerifyTextChunks(all.data(), all.size(), boff, blen, got, arena.data(), arena.size(), valid) ==
          Error::NO_ERROR_LBF);
    CHECK(valid == "1011");
    CHECK(got[3].m_size == 777 && std::memcmp(arena.data() + 3 * 65536, data.data() + 3 * 65536, 777) == 0);
  }

  // multi-file EncodeFile (Encoder.cpp:17-102): every file of m_files, an empty
  // one included (no chunks), keyed by name; the hashes equal the batch path's
  {
    const std::vector<std::pair<std::string, size_t>> files = {
        {dir + "/c.bin", 2 * 65536 + 56}, {dir + "/a.bin", 100000}, {dir + "/b.bin", 0}};
    Encoder::ToEncode me;
    me.m_chunksize = 65536;
    std::vector<std::vector<U8>> bytes;
    for (size_t k = 0; k < files.size(); ++k) {
      bytes.push_back(pattern(files[k].second, 20 + (U32)k));
      FILE* g = std::fopen(files[k].first.c_str(), "wb");
      if (!bytes.back().empty()) std::fwrite(bytes.back().data(), 1, bytes.back().size(), g);
      std::fclose(g);
      me.m_files.push_back(files[k].first);
    }
    FloodFile mf;
    CHECK(Encoder::EncodeFile(me, mf) == Error::NO_ERROR_LBF);
    CHECK(mf.m_files.size() == 3);
    for (size_t k = 0; k < files.size(); ++k) {
      const FloodFile::FileSPtr& fe = mf.m_files[files[k].first];
      const size_t n = (files[k].second + 65535) / 65536;
      CHECK(fe && fe->m_size == files[k].second && fe->m_chunks.size() == n);
      std::vector<U64> o(n);
      std::vector<U32> z(n);
      for (size_t i = 0; i < n; ++i) {
        o[i] = 65536ull * i;
        z[i] = (U32)std::min<size_t>(65536, files[k].second - 65536 * i);
      }
      V_String want;
      if (n) CHECK(Encoder::Base64EncodeBatch(bytes[k].data(), bytes[k].size(), o.data(), z.data(), n, want) ==
                   Error::NO_ERROR_LBF);
      for (size_t i = 0; fe && i < n && i < fe->m_chunks.size() && i < want.size(); ++i) {
        CHECK(fe->m_chunks[i].m_index == i && fe->m_chunks[i].m_size == z[i] && fe->m_chunks[i].m_hash == want[i]);
      }
    }
    // the same three files through the resume verify, batched over files
    // (Flood.cpp:220-299): intact -> all '1'; then c.bin loses its tail,
    // a.bin's second chunk gets a flipped byte, b.bin stays empty
    {
      FloodFileSPtr mff(new FloodFile(mf));
      Flood mv;
      CHECK(mv.Initialize(mff) == Error::NO_ERROR_LBF);
      CHECK(mv.m_runtimefiles[files[0].first].m_chunkmap == "111");
      CHECK(mv.m_runtimefiles[files[1].first].m_chunkmap == "11");
      CHECK(mv.m_runtimefiles[files[2].first].m_chunkmap.empty());
      CHECK(mv.m_chunkstodownload.empty());
      FILE* g = std::fopen(files[0].first.c_str(), "wb");
      std::fwrite(bytes[0].data(), 1, 65536 + 10, g);
      std::fclose(g);
      std::vector<U8> a = bytes[1];
      a[65536 + 3] ^= 0x20;
      g = std::fopen(files[1].first.c_str(), "wb");
      std::fwrite(a.data(), 1, a.size(), g);
      std::fclose(g);
      Flood mv2;
      CHECK(mv2.Initialize(mff) == Error::NO_ERROR_LBF);
      CHECK(mv2.m_runtimefiles[files[0].first].m_chunkmap == "100");
      CHECK(mv2.m_runtimefiles[files[1].first].m_chunkmap == "10");
      CHECK(mv2.m_chunkstodownload.size() == 3);
      // restore c.bin and a.bin for what follows
      g = std::fopen(files[0].first.c_str(), "wb");
      std::fwrite(bytes[0].data(), 1, bytes[0].size(), g);
      std::fclose(g);
      g = std::fopen(files[1].first.c_str(), "wb");
      std::fwrite(bytes[1].data(), 1, bytes[1].size(), g);
      std::fclose(g);
    }
    // the batched verify fails once (one-shot injected fault at the context's
    // first group): each file is verified on its own, every retry succeeds, so
    // Initialize reports success with complete chunkmaps
    {
      setenv("LBF_TEST_FAULT_GROUP", "0", 1);
      lbf_ctx* fctx = nullptr;
      const int made = lbf_ctx_create(1u, &fctx);
      unsetenv("LBF_TEST_FAULT_GROUP");
      CHECK(made == LBF_OK);
      if (made == LBF_OK) {
        FloodFileSPtr mff(new FloodFile(mf));
        Flood mv3;
        mv3.m_ctx = fctx;
        CHECK(mv3.Initialize(mff) == Error::NO_ERROR_LBF);
        CHECK(mv3.m_runtimefiles[files[0].first].m_chunkmap == "111");
        CHECK(mv3.m_runtimefiles[files[1].first].m_chunkmap == "11");
        CHECK(mv3.m_runtimefiles.size() == 3 && mv3.m_chunkstodownload.empty());
        CHECK(mv3.m_totalbytes == files[0].second + files[1].second + files[2].second);
        lbf_ctx_destroy(fctx);
      }
    }
    // a missing file: the call fails and the output is left as it was (:45-47, :96-99)
    me.m_files.push_back(dir + "/missing.bin");
    FloodFile untouched;
    CHECK(Encoder::EncodeFile(me, untouched) == Error::UNKNOWN_ERROR_LBF);
    CHECK(untouched.m_files.empty());
  }

  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed (last error: %s)\n", g_fail, Encoder::LastError());
    return 1;
  }
  std::printf("gpu_tests OK\n");
  return 0;
}
