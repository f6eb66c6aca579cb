// Encoder.cpp -- libBitFlood::Encoder on MI355X.
//
// EncodeFile / Base64Encode keep the reference's signatures and results
// (/root/reference/cpp/src/Encoder.cpp:17-120); the per-chunk
// fread -> Crypto++ SHA -> BaseN_Encoder loop becomes one pipelined batch per
// file: pread into pinned staging, H2D, the gfx950 chunk-hash kernel, D2H of
// 20-byte digests, then the 27-char rendering on the host.
#include "libBitFlood/Encoder.H"

#include <sys/stat.h>

#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "lbf_hash.h"

namespace libBitFlood {
namespace Encoder {

namespace {

std::mutex g_mu;
// Shared: SetDeviceMask drops the process's reference, and calls still running
// on other threads keep theirs until they return.
std::shared_ptr<lbf_ctx> g_ctx;
U32 g_mask = 0;
thread_local std::string t_err;

Error::ErrorCode fail(const std::string& where) {
  const char* e = lbf_last_error();
  t_err = where + ": " + (e ? e : "");
  return Error::UNKNOWN_ERROR_LBF;
}

std::string b64(const U8* digest) {
  char s[28];
  lbf_b64_27(digest, s);
  return std::string(s, 27);
}

struct CtxReaper {
  ~CtxReaper() {
    std::lock_guard<std::mutex> lock(g_mu);
    g_ctx.reset();
  }
} g_reaper;

}  // namespace

std::shared_ptr<lbf_ctx> SharedContext() {
  std::lock_guard<std::mutex> lock(g_mu);
  if (!g_ctx) {
    lbf_ctx* c = nullptr;
    if (lbf_ctx_create(g_mask, &c) == LBF_OK) g_ctx.reset(c, lbf_ctx_destroy);
    else fail("lbf_ctx_create");
  }
  return g_ctx;
}

lbf_ctx* Context() { return SharedContext().get(); }

Error::ErrorCode SetDeviceMask(U32 i_mask) {
  std::shared_ptr<lbf_ctx> old;
  {
    std::lock_guard<std::mutex> lock(g_mu);
    old.swap(g_ctx);
    g_mask = i_mask;
  }
  return Error::NO_ERROR_LBF;  // `old` is destroyed here unless a call still holds it
}

const char* LastError() { return t_err.c_str(); }

Error::ErrorCode Base64Encode(const U8* i_data, U32 i_size, std::string& o_string) {
  const std::shared_ptr<lbf_ctx> held = SharedContext();  // alive for the whole call
  lbf_ctx* ctx = held.get();
  if (!ctx) return Error::UNKNOWN_ERROR_LBF;
  U8 d[20];
  if (lbf_sha1_one(ctx, i_data, i_size, d) != LBF_OK) return fail("Base64Encode");
  o_string = b64(d);
  return Error::NO_ERROR_LBF;
}

Error::ErrorCode HashChunks(const U8* i_base, U64 i_len, const U64* i_offsets, const U32* i_sizes, U64 i_n,
                            V_U8& o_digests) {
  o_digests.assign(i_n * 20, 0);
  if (i_n == 0) return Error::NO_ERROR_LBF;
  const std::shared_ptr<lbf_ctx> held = SharedContext();  // alive for the whole call
  lbf_ctx* ctx = held.get();
  if (!ctx) return Error::UNKNOWN_ERROR_LBF;
  if (lbf_sha1_batch(ctx, i_base, i_len, i_offsets, i_sizes, i_n, o_digests.data(), LBF_HOST_PTR) != LBF_OK)
    return fail("HashChunks");
  return Error::NO_ERROR_LBF;
}

Error::ErrorCode Base64EncodeBatch(const U8* i_base, U64 i_len, const U64* i_offsets, const U32* i_sizes, U64 i_n,
                                   V_String& o_hashes) {
  V_U8 d;
  const Error::ErrorCode rc = HashChunks(i_base, i_len, i_offsets, i_sizes, i_n, d);
  if (rc != Error::NO_ERROR_LBF) return rc;
  o_hashes.resize(i_n);
  for (U64 i = 0; i < i_n; ++i) o_hashes[i] = b64(&d[20 * i]);
  return Error::NO_ERROR_LBF;
}

// Encoder.cpp:17-102.  The reference hashes its files one after another; here
// every existing file's chunks go to the GPU in ONE pipelined batch
// (lbf_files_ranges), because each chunk's serial SHA-1 chain costs the same
// whatever the batch: per-file calls would pay ≈3 ms per file at 256 KiB
// chunks.  Results and error behaviour are the reference's.
Error::ErrorCode EncodeFile(const ToEncode& i_toencode, FloodFile& o_floodfile) {
  Error::ErrorCode ret = Error::NO_ERROR_LBF;
  FloodFile toReturn;
  if (i_toencode.m_files.empty() || i_toencode.m_chunksize == 0) {  // Encoder.cpp:24-31
    t_err = "EncodeFile: empty file list or zero chunk size";
    ret = Error::UNKNOWN_ERROR_LBF;
  } else {
    const std::shared_ptr<lbf_ctx> held = SharedContext();  // alive for the whole call
    lbf_ctx* ctx = held.get();
    if (!ctx) return Error::UNKNOWN_ERROR_LBF;
    const U64 cs = i_toencode.m_chunksize;
    std::vector<const char*> paths;  // files that exist, in the given order
    std::vector<U64> size_of, first_of;
    V_U64 offs;
    V_U32 sizes, file_of;
    for (const std::string& path : i_toencode.m_files) {  // in the given order, like :40
      struct stat st;
      if (stat(path.c_str(), &st) != 0 || S_ISDIR(st.st_mode)) {
        t_err = "EncodeFile: cannot open " + path;  // fopen failed: :45-47, keep going
        ret = Error::UNKNOWN_ERROR_LBF;
        continue;
      }
      const U64 size = (U64)st.st_size;
      const U64 n = (size + cs - 1) / cs;  // the fread loop's chunk count (:54-72)
      const U32 f = (U32)paths.size();
      paths.push_back(path.c_str());
      size_of.push_back(size);
      first_of.push_back(offs.size());
      for (U64 i = 0; i < n; ++i) {
        offs.push_back(i * cs);
        sizes.push_back((U32)std::min<U64>(cs, size - i * cs));
        file_of.push_back(f);
      }
    }
    V_U8 digests(offs.size() * 20);
    if (!offs.empty() && lbf_files_ranges(ctx, paths.data(), (U32)paths.size(), file_of.data(), offs.data(),
                                          sizes.data(), offs.size(), nullptr, digests.data()) != LBF_OK) {
      fail("EncodeFile");
      ret = Error::UNKNOWN_ERROR_LBF;
    } else {
      for (size_t f = 0; f < paths.size(); ++f) {
        const U64 first = first_of[f], n = (f + 1 < paths.size() ? first_of[f + 1] : offs.size()) - first;
        FloodFile::FileSPtr file(new FloodFile::File());
        file->m_name = paths[f];
        file->m_size = size_of[f];  // 64-bit; the reference's U32 wraps at 4 GiB (:76)
        file->m_chunks.resize(n);
        for (U64 i = 0; i < n; ++i) {
          FloodFile::Chunk& c = file->m_chunks[i];
          c.m_index = (U32)i;
          c.m_size = sizes[first + i];
          c.m_weight = 0;
          c.m_hash = b64(&digests[20 * (first + i)]);
        }
        toReturn.m_files[paths[f]] = file;
      }
    }
    for (const ToEncode::Tracker& t : i_toencode.m_trackers) {  // :83-93
      FloodFile::TrackerInfo ti;
      ti.m_host = t.first;
      ti.m_port = t.second;
      toReturn.m_trackers.push_back(ti);
    }
  }
  if (ret == Error::NO_ERROR_LBF) o_floodfile = toReturn;  // :96-99
  return ret;
}

}  // namespace Encoder
}  // namespace libBitFlood
