// Flood.cpp -- the verify paths of the reference's Flood / ChunkMethodHandler,
// batched onto the GPU (see include/libBitFlood/Flood.H for the mapping).
#include "libBitFlood/Flood.H"

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <system_error>
#include <thread>
#include <vector>

#include "lbf_hash.h"
#include "libBitFlood/Encoder.H"

namespace libBitFlood {

namespace {

// 27-char string -> 20 raw bytes.  A string that is not canonical base64-27
// can never equal a computed hash, so it yields ok = false (verdict 0 without
// hashing), exactly what the reference's string compare gives.
bool decode_hash(const std::string& s, U8* out) {
  return lbf_b64_27_decode(s.data(), s.size(), out) == LBF_OK;
}

// Run f(k) for k in [0, n) on up to `threads` threads (file reads/writes of a
// batch: one thread moves ~2-3 GB/s through the page cache).
template <class F>
void parallel_for(size_t n, unsigned threads, F f) {
  threads = (unsigned)std::min<size_t>(threads, n);
  if (threads <= 1) {
    for (size_t k = 0; k < n; ++k) f(k);
    return;
  }
  std::atomic<size_t> next{0};
  auto pull = [&] {
    for (size_t k; (k = next++) < n;) f(k);
  };
  // helpers plus the calling thread; a helper that cannot be started leaves
  // its share to the others (a joinable thread must never be destroyed)
  std::vector<std::thread> th;
  for (unsigned t = 1; t < threads; ++t) {
    try {
      th.emplace_back(pull);
    } catch (const std::system_error&) {
      break;
    }
  }
  pull();
  for (auto& t : th) t.join();
}

unsigned io_threads() {
  const char* v = getenv("LBF_COPY_THREADS");
  const long n = v && *v ? strtol(v, nullptr, 10) : 8;
  return (unsigned)std::max(1L, std::min(64L, n));
}

}  // namespace

std::shared_ptr<lbf_ctx> Flood::Ctx() const {
  if (m_ctx) return std::shared_ptr<lbf_ctx>(m_ctx, [](lbf_ctx*) {});  // the caller owns it
  return Encoder::SharedContext();
}

std::string Flood::PathOf(const std::string& i_name) const {
  if (m_rootdir.empty() || (!i_name.empty() && i_name[0] == '/')) return i_name;
  return m_rootdir + "/" + i_name;
}

Error::ErrorCode Flood::Initialize(FloodFileSPtr& i_floodfile) {
  m_floodfile = i_floodfile;
  return SetupFilesAndChunks();  // Flood.cpp:25-35
}

// Flood.cpp:243-257: chunk k of the vector (sorted by index in FromXML) starts
// where chunk k-1 ended.  64-bit offsets; the reference's U32 next_offset
// wraps past 4 GiB.  False when the indices are not 0..n-1 exactly once (the
// reference asserts, Flood.cpp:253-254).
bool Flood::LayoutChunks(const FloodFile::File& i_file, V_U64& o_offsets) {
  const U64 n = i_file.m_chunks.size();
  o_offsets.assign(n, 0);
  std::vector<bool> seen(n, false);
  U64 next = 0;
  for (U64 k = 0; k < n; ++k) {
    const FloodFile::Chunk& c = i_file.m_chunks[k];
    if (c.m_index >= n || seen[c.m_index]) return false;
    seen[c.m_index] = true;
    o_offsets[c.m_index] = next;
    next += c.m_size;
  }
  return true;
}

// Flood.cpp:220-299.  Per file: lay the chunks out back to back in index
// order; then hash every chunk of every file that exists on disk in ONE
// batched verify (lbf_files_ranges).  The reference does fseek + malloc +
// fread + Base64Encode + strcmp per chunk, file after file.  If the batch
// fails (a HIP error, no memory), each file is verified on its own, and a file
// whose own call fails too is left out of m_runtimefiles and m_totalbytes.
Error::ErrorCode Flood::SetupFilesAndChunks() {
  m_totalbytes = 0;
  m_runtimefiles.clear();
  m_chunkstodownload.clear();
  if (!m_floodfile) return Error::UNKNOWN_ERROR_LBF;
  const std::shared_ptr<lbf_ctx> held = Ctx();  // alive for the whole call
  lbf_ctx* ctx = held.get();
  if (!ctx) return Error::UNKNOWN_ERROR_LBF;
  Error::ErrorCode ret = Error::NO_ERROR_LBF;
  std::vector<RuntimeFile> rtfs;
  std::vector<std::string> paths;
  std::vector<U64> first_of;
  V_U64 offs;
  V_U32 sizes, file_of;
  V_U8 expected;
  std::vector<U8> decodable;
  for (const auto& kv : m_floodfile->m_files) {
    const FloodFile::FileSPtr& file = kv.second;
    RuntimeFile rtf;
    const U64 n = file->m_chunks.size();
    rtf.m_chunkmap.assign(n, '0');
    rtf.m_file = file;
    if (!LayoutChunks(*file, rtf.m_chunkoffsets)) {
      ret = Error::UNKNOWN_ERROR_LBF;
      continue;
    }
    first_of.push_back(offs.size());
    for (U64 k = 0; k < n; ++k) {
      const FloodFile::Chunk& c = file->m_chunks[k];
      offs.push_back(rtf.m_chunkoffsets[c.m_index]);
      sizes.push_back(c.m_size);
      file_of.push_back((U32)paths.size());
      expected.resize(expected.size() + 20, 0);
      decodable.push_back(decode_hash(c.m_hash, &expected[expected.size() - 20]) ? 1 : 0);
    }
    paths.push_back(PathOf(file->m_name));
    rtfs.push_back(rtf);
  }
  first_of.push_back(offs.size());
  V_U8 verdicts(offs.size(), 0);
  std::vector<U8> file_ok(rtfs.size(), 1);
  std::vector<const char*> cpaths;
  for (const std::string& p : paths) cpaths.push_back(p.c_str());
  if (!offs.empty() && lbf_files_ranges(ctx, cpaths.data(), (U32)cpaths.size(), file_of.data(), offs.data(),
                                        sizes.data(), offs.size(), expected.data(), verdicts.data()) != LBF_OK) {
    // One file at a time; the call fails only if some file's own call fails
    // too (a batch failure the retries recover from leaves complete state).
    for (size_t f = 0; f < rtfs.size(); ++f) {
      const U64 b = first_of[f], e = first_of[f + 1];
      if (b == e) continue;
      const U32 zero = 0;
      V_U32 fo(e - b, zero);
      file_ok[f] = lbf_files_ranges(ctx, &cpaths[f], 1, fo.data(), offs.data() + b, sizes.data() + b, e - b,
                                    expected.data() + 20 * b, verdicts.data() + b) == LBF_OK;
      if (!file_ok[f]) ret = Error::UNKNOWN_ERROR_LBF;
    }
  }
  for (size_t f = 0; f < rtfs.size(); ++f) {
    if (!file_ok[f]) continue;
    RuntimeFile& rtf = rtfs[f];
    const FloodFile::FileSPtr& file = rtf.m_file;
    const U64 first = first_of[f];
    m_totalbytes += file->m_size;
    for (U64 k = 0; k < file->m_chunks.size(); ++k) {
      const U32 idx = file->m_chunks[k].m_index;
      if (verdicts[first + k] && decodable[first + k]) rtf.m_chunkmap[idx] = '1';
      if (rtf.m_chunkmap[idx] == '0') m_chunkstodownload.insert(P_ChunkKey(file->m_name, idx));
    }
    m_runtimefiles[file->m_name] = rtf;
  }
  return ret;
}

// ChunkMethods.cpp:89-135 (seeder): read the chunk at its offset and send it
// only if it still hashes to the flood-file value.
Error::ErrorCode Flood::ReadVerifiedChunk(const std::string& i_filename, U32 i_chunkindex, V_U8& o_data,
                                          bool& o_valid) {
  o_valid = false;
  o_data.clear();
  auto it = m_runtimefiles.find(i_filename);
  if (it == m_runtimefiles.end() || i_chunkindex >= it->second.m_file->m_chunks.size())
    return Error::NO_ERROR_LBF;  // unknown file/chunk: nothing sent
  const FloodFile::Chunk& chunk = it->second.m_file->m_chunks[i_chunkindex];
  const U64 off = it->second.m_chunkoffsets[i_chunkindex];
  const int fd = open(PathOf(i_filename).c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return Error::NO_ERROR_LBF;
  o_data.resize(chunk.m_size);
  U64 got = 0;
  while (got < chunk.m_size) {
    const ssize_t r = pread(fd, o_data.data() + got, chunk.m_size - got, (off_t)(off + got));
    if (r <= 0) break;
    got += (U64)r;
  }
  close(fd);
  U8 expected[20];
  if (got != chunk.m_size || !decode_hash(chunk.m_hash, expected)) {
    o_data.clear();
    return Error::NO_ERROR_LBF;
  }
  const std::shared_ptr<lbf_ctx> held = Ctx();  // alive for the whole call
  lbf_ctx* ctx = held.get();
  if (!ctx) return Error::UNKNOWN_ERROR_LBF;
  const U64 zero = 0;
  const U32 sz = chunk.m_size;
  U8 verdict = 0;
  static const U8 kEmpty = 0;
  if (lbf_verify_batch(ctx, sz ? o_data.data() : &kEmpty, sz, &zero, &sz, 1, expected, &verdict, LBF_HOST_PTR) !=
      LBF_OK)
    return Error::UNKNOWN_ERROR_LBF;
  o_valid = verdict != 0;
  if (!o_valid) o_data.clear();
  return Error::NO_ERROR_LBF;
}

// ChunkMethods.cpp:137-225 (receiver): size check, verify on the GPU, write
// at the chunk's offset, mark it '1' and stop wanting it.  (Broadcasting
// NotifyHaveChunk and the in-flight bookkeeping belong to the peer loop.)
Error::ErrorCode Flood::ReceiveChunk(const std::string& i_filename, U32 i_chunkindex, const U8* i_data, U32 i_size,
                                     bool& o_accepted) {
  o_accepted = false;
  auto it = m_runtimefiles.find(i_filename);
  if (it == m_runtimefiles.end() || i_chunkindex >= it->second.m_file->m_chunks.size())
    return Error::NO_ERROR_LBF;
  RuntimeFile& rtf = it->second;
  const FloodFile::Chunk& chunk = rtf.m_file->m_chunks[i_chunkindex];
  if (chunk.m_size != i_size) return Error::NO_ERROR_LBF;  // :156
  U8 expected[20];
  if (!decode_hash(chunk.m_hash, expected)) return Error::NO_ERROR_LBF;
  const std::shared_ptr<lbf_ctx> held = Ctx();  // alive for the whole call
  lbf_ctx* ctx = held.get();
  if (!ctx) return Error::UNKNOWN_ERROR_LBF;
  const U64 zero = 0;
  U8 verdict = 0;
  static const U8 kEmpty = 0;
  if (lbf_verify_batch(ctx, i_size ? i_data : &kEmpty, i_size, &zero, &i_size, 1, expected, &verdict,
                       LBF_HOST_PTR) != LBF_OK)
    return Error::UNKNOWN_ERROR_LBF;
  if (!verdict) return Error::NO_ERROR_LBF;  // bad chunk silently dropped (:167)
  const std::string path = PathOf(i_filename);
  FILE* f = fopen(path.c_str(), "r+b");  // :169-173
  if (!f) f = fopen(path.c_str(), "w+b");
  if (!f) return Error::NO_ERROR_LBF;
  bool ok = fseeko(f, (off_t)rtf.m_chunkoffsets[i_chunkindex], SEEK_SET) == 0;
  if (ok) ok = fwrite(i_data, 1, i_size, f) == i_size;
  fclose(f);
  if (!ok) return Error::NO_ERROR_LBF;
  rtf.m_chunkmap[i_chunkindex] = '1';  // :181-185
  m_chunkstodownload.erase(P_ChunkKey(it->first, i_chunkindex));
  o_accepted = true;
  return Error::NO_ERROR_LBF;
}

Error::ErrorCode Flood::ReadVerifiedChunks(const std::vector<P_ChunkKey>& i_keys, V_U8& o_arena, V_U64& o_offsets,
                                           std::string& o_valid) {
  const size_t n = i_keys.size();
  o_offsets.assign(n, 0);
  o_valid.assign(n, '0');
  V_U32 sizes(n, 0);
  V_U8 expected(n * 20, 0);
  std::vector<int> ok(n, 0);
  U64 total = 0;
  for (size_t k = 0; k < n; ++k) {
    auto it = m_runtimefiles.find(i_keys[k].first);
    if (it == m_runtimefiles.end() || i_keys[k].second >= it->second.m_file->m_chunks.size()) continue;
    const FloodFile::Chunk& c = it->second.m_file->m_chunks[i_keys[k].second];
    if (!decode_hash(c.m_hash, &expected[20 * k])) continue;
    o_offsets[k] = total;
    sizes[k] = c.m_size;
    total += (c.m_size + 15) & ~15ull;  // keep every chunk 16-byte aligned in the arena
    ok[k] = 1;
  }
  // grown, never cleared: every byte the verify reads is pread first
  if (o_arena.size() < std::max<U64>(total, 1)) o_arena.resize(std::max<U64>(total, 1));
  // one open per file, pread per chunk (ChunkMethods.cpp:105-115 fopen/fread per request)
  std::map<std::string, int> fds;
  for (size_t k = 0; k < n; ++k)
    if (ok[k] && !fds.count(i_keys[k].first))
      fds[i_keys[k].first] = open(PathOf(i_keys[k].first).c_str(), O_RDONLY | O_CLOEXEC);
  parallel_for(n, io_threads(), [&](size_t k) {
    if (!ok[k]) return;
    const int fd = fds.find(i_keys[k].first)->second;
    const off_t off = (off_t)m_runtimefiles.find(i_keys[k].first)->second.m_chunkoffsets[i_keys[k].second];
    U64 got = 0;
    while (fd >= 0 && got < sizes[k]) {
      const ssize_t r = pread(fd, &o_arena[o_offsets[k]] + got, sizes[k] - got, off + (off_t)got);
      if (r <= 0) break;
      got += (U64)r;
    }
    if (got != sizes[k]) ok[k] = 0;
  });
  for (auto& f : fds)
    if (f.second >= 0) close(f.second);
  std::vector<U64> voff;
  std::vector<U32> vsz;
  std::vector<U8> vexp;
  std::vector<size_t> which;
  for (size_t k = 0; k < n; ++k) {
    if (!ok[k]) continue;
    which.push_back(k);
    voff.push_back(o_offsets[k]);
    vsz.push_back(sizes[k]);
    vexp.insert(vexp.end(), &expected[20 * k], &expected[20 * k] + 20);
  }
  if (which.empty()) return Error::NO_ERROR_LBF;
  const std::shared_ptr<lbf_ctx> held = Ctx();  // alive for the whole call
  lbf_ctx* ctx = held.get();
  if (!ctx) return Error::UNKNOWN_ERROR_LBF;
  std::vector<U8> verdict(which.size(), 0);
  if (lbf_verify_batch(ctx, &o_arena[0], o_arena.size(), &voff[0], &vsz[0], which.size(), &vexp[0], &verdict[0],
                       LBF_HOST_PTR) != LBF_OK)
    return Error::UNKNOWN_ERROR_LBF;
  for (size_t j = 0; j < which.size(); ++j)
    if (verdict[j]) o_valid[which[j]] = '1';
  return Error::NO_ERROR_LBF;
}

Error::ErrorCode Flood::VerifyChunks(const U8* i_arena, U64 i_arena_len, const std::vector<ChunkArrival>& i_chunks,
                                     std::string& o_valid) {
  const size_t n = i_chunks.size();
  o_valid.assign(n, '0');
  std::vector<U64> voff;
  std::vector<U32> vsz;
  std::vector<U8> vexp;
  std::vector<size_t> which;
  for (size_t k = 0; k < n; ++k) {
    const ChunkArrival& a = i_chunks[k];
    auto it = m_runtimefiles.find(a.m_filename);
    if (it == m_runtimefiles.end() || a.m_index >= it->second.m_file->m_chunks.size()) continue;
    const FloodFile::Chunk& c = it->second.m_file->m_chunks[a.m_index];
    if (c.m_size != a.m_size) continue;  // ChunkMethods.cpp:156
    if (a.m_offset > i_arena_len || a.m_size > i_arena_len - a.m_offset) continue;
    U8 e[20];
    if (!decode_hash(c.m_hash, e)) continue;
    which.push_back(k);
    voff.push_back(a.m_offset);
    vsz.push_back(a.m_size);
    vexp.insert(vexp.end(), e, e + 20);
  }
  if (which.empty()) return Error::NO_ERROR_LBF;
  const std::shared_ptr<lbf_ctx> held = Ctx();  // alive for the whole call
  lbf_ctx* ctx = held.get();
  if (!ctx) return Error::UNKNOWN_ERROR_LBF;
  std::vector<U8> verdict(which.size(), 0);
  static const U8 kEmpty = 0;
  if (lbf_verify_batch(ctx, i_arena_len ? i_arena : &kEmpty, i_arena_len, &voff[0], &vsz[0], which.size(), &vexp[0],
                       &verdict[0], LBF_HOST_PTR) != LBF_OK)
    return Error::UNKNOWN_ERROR_LBF;
  for (size_t j = 0; j < which.size(); ++j)
    if (verdict[j]) o_valid[which[j]] = '1';
  return Error::NO_ERROR_LBF;
}

// ChunkMethods.cpp:116-123 and the encode of its SendChunk payload
// (XmlRpcValue::binaryToXml), both on the GPU from one device copy: chunk k's
// base64 text lands at o_text + i_text_offsets[k] (lbf_b64_put_length of its
// size) whatever its verdict.  Chunks VerifyChunks would skip stay '0' and get
// no text.
Error::ErrorCode Flood::VerifyEncodeChunks(const U8* i_arena, U64 i_arena_len, const std::vector<ChunkArrival>& i_chunks,
                                           std::string& o_valid, char* o_text, U64 i_text_len,
                                           const V_U64& i_text_offsets) {
  const size_t n = i_chunks.size();
  o_valid.assign(n, '0');
  if (i_text_offsets.size() != n) return Error::UNKNOWN_ERROR_LBF;
  V_U64 voff, toff;
  V_U32 vsz;
  V_U8 vexp;
  std::vector<size_t> which;
  for (size_t k = 0; k < n; ++k) {
    const ChunkArrival& a = i_chunks[k];
    auto it = m_runtimefiles.find(a.m_filename);
    if (it == m_runtimefiles.end() || a.m_index >= it->second.m_file->m_chunks.size()) continue;
    const FloodFile::Chunk& c = it->second.m_file->m_chunks[a.m_index];
    if (c.m_size != a.m_size) continue;
    if (a.m_offset > i_arena_len || a.m_size > i_arena_len - a.m_offset) continue;
    const U64 tl = lbf_b64_put_length(a.m_size);
    if (i_text_offsets[k] > i_text_len || tl > i_text_len - i_text_offsets[k]) continue;
    U8 e[20];
    if (!decode_hash(c.m_hash, e)) continue;
    which.push_back(k);
    voff.push_back(a.m_offset);
    vsz.push_back(a.m_size);
    toff.push_back(i_text_offsets[k]);
    vexp.insert(vexp.end(), e, e + 20);
  }
  if (which.empty()) return Error::NO_ERROR_LBF;
  const std::shared_ptr<lbf_ctx> held = Ctx();  // alive for the whole call
  lbf_ctx* ctx = held.get();
  if (!ctx) return Error::UNKNOWN_ERROR_LBF;
  std::vector<U8> verdict(which.size(), 0);
  static const U8 kEmpty = 0;
  if (lbf_verify_encode_b64_batch(ctx, i_arena_len ? i_arena : &kEmpty, i_arena_len, &voff[0], &vsz[0], which.size(),
                                  &vexp[0], &verdict[0], o_text, i_text_len, &toff[0]) != LBF_OK)
    return Error::UNKNOWN_ERROR_LBF;
  for (size_t j = 0; j < which.size(); ++j)
    if (verdict[j]) o_valid[which[j]] = '1';
  return Error::NO_ERROR_LBF;
}

// ChunkMethods.cpp:137-167 from the wire form: the base64 decode of the
// SendChunk payload (XmlRpcValue.cpp:417-436) and the verify, both on the GPU.
// Chunks whose file or index the flood does not know, whose output slot does
// not fit the arena, or whose flood-file hash does not decode stay '0'.
Error::ErrorCode Flood::VerifyTextChunks(const char* i_text, U64 i_text_len, const V_U64& i_text_offsets,
                                         const V_U32& i_text_lengths, std::vector<ChunkArrival>& io_chunks,
                                         U8* o_arena, U64 i_arena_len, std::string& o_valid) {
  const size_t n = io_chunks.size();
  o_valid.assign(n, '0');
  if (i_text_offsets.size() != n || i_text_lengths.size() != n) return Error::UNKNOWN_ERROR_LBF;
  V_U64 toff, ooff;
  V_U32 tlen, esz;
  V_U8 vexp;
  std::vector<size_t> which;
  for (size_t k = 0; k < n; ++k) {
    ChunkArrival& a = io_chunks[k];
    a.m_size = 0;
    auto it = m_runtimefiles.find(a.m_filename);
    if (it == m_runtimefiles.end() || a.m_index >= it->second.m_file->m_chunks.size()) continue;
    const FloodFile::Chunk& c = it->second.m_file->m_chunks[a.m_index];
    if (a.m_offset > i_arena_len || c.m_size > i_arena_len - a.m_offset) continue;
    if (i_text_offsets[k] > i_text_len || i_text_lengths[k] > i_text_len - i_text_offsets[k]) continue;
    U8 e[20];
    if (!decode_hash(c.m_hash, e)) continue;
    which.push_back(k);
    toff.push_back(i_text_offsets[k]);
    tlen.push_back(i_text_lengths[k]);
    ooff.push_back(a.m_offset);
    esz.push_back(c.m_size);
    vexp.insert(vexp.end(), e, e + 20);
  }
  if (which.empty()) return Error::NO_ERROR_LBF;
  const std::shared_ptr<lbf_ctx> held = Ctx();  // alive for the whole call
  lbf_ctx* ctx = held.get();
  if (!ctx) return Error::UNKNOWN_ERROR_LBF;
  std::vector<U8> verdict(which.size(), 0);
  V_U32 got(which.size(), 0);
  if (lbf_b64_verify_batch(ctx, i_text, i_text_len, &toff[0], &tlen[0], which.size(), &esz[0], &vexp[0], o_arena,
                           i_arena_len, &ooff[0], &got[0], &verdict[0]) != LBF_OK)
    return Error::UNKNOWN_ERROR_LBF;
  for (size_t j = 0; j < which.size(); ++j) {
    // the decoded length, as DecodeSendChunk would report it; a text longer
    // than the chunk is rejected (ChunkMethods.cpp:156) and writes nothing
    io_chunks[which[j]].m_size = got[j] <= esz[j] ? got[j] : 0;
    if (verdict[j]) o_valid[which[j]] = '1';
  }
  return Error::NO_ERROR_LBF;
}

Error::ErrorCode Flood::ReceiveChunks(const U8* i_arena, U64 i_arena_len, const std::vector<ChunkArrival>& i_chunks,
                                      std::string& o_accepted) {
  o_accepted.assign(i_chunks.size(), '0');
  std::string valid;
  const Error::ErrorCode rc = VerifyChunks(i_arena, i_arena_len, i_chunks, valid);
  if (rc != Error::NO_ERROR_LBF) return rc;
  return WriteChunks(i_arena, i_chunks, valid, o_accepted);
}

// ChunkMethods.cpp:169-185: write each chunk whose verdict is '1' at its
// offset, then mark it '1' and drop it from the download set.
Error::ErrorCode Flood::WriteChunks(const U8* i_arena, const std::vector<ChunkArrival>& i_chunks,
                                    const std::string& i_valid, std::string& o_accepted) {
  const size_t n = i_chunks.size();
  o_accepted.assign(n, '0');
  if (i_valid.size() != n) return Error::UNKNOWN_ERROR_LBF;
  const std::string& valid = i_valid;
  std::vector<size_t> which;
  for (size_t k = 0; k < n; ++k)
    if (valid[k] == '1') which.push_back(k);
  if (which.empty()) return Error::NO_ERROR_LBF;
  // write the accepted chunks: one open per file (fopen "r+b" else "w+b", :169-173)
  std::map<std::string, int> fds;
  for (size_t k : which) {
    const std::string& name = i_chunks[k].m_filename;
    if (!fds.count(name)) fds[name] = open(PathOf(name).c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0644);
  }
  std::vector<U8> written(which.size(), 0);
  parallel_for(which.size(), io_threads(), [&](size_t j) {
    const ChunkArrival& a = i_chunks[which[j]];
    const int fd = fds.find(a.m_filename)->second;
    if (fd < 0) return;
    const off_t off = (off_t)m_runtimefiles.find(a.m_filename)->second.m_chunkoffsets[a.m_index];
    U64 put = 0;
    while (put < a.m_size) {
      const ssize_t w = pwrite(fd, i_arena + a.m_offset + put, a.m_size - put, off + (off_t)put);
      if (w <= 0) break;
      put += (U64)w;
    }
    written[j] = put == a.m_size;
  });
  for (size_t j = 0; j < which.size(); ++j) {
    if (!written[j]) continue;
    const ChunkArrival& a = i_chunks[which[j]];
    m_runtimefiles[a.m_filename].m_chunkmap[a.m_index] = '1';  // :181-185
    m_chunkstodownload.erase(P_ChunkKey(a.m_filename, a.m_index));
    o_accepted[which[j]] = '1';
  }
  for (auto& f : fds)
    if (f.second >= 0) close(f.second);
  return Error::NO_ERROR_LBF;
}

}  // namespace libBitFlood
