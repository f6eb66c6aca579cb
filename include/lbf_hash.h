/*
 * lbf_hash.h -- C ABI of the MI355X chunk-hash path for bitflood.
 *
 * This is the drop-in boundary beneath the reference's C++ entry points
 *   Error::ErrorCode libBitFlood::Encoder::Base64Encode(const U8*, U32, std::string&)
 *       (/root/reference/cpp/src/Encoder.H:28, Encoder.cpp:107-120)
 *   Error::ErrorCode libBitFlood::Encoder::EncodeFile(const ToEncode&, FloodFile&)
 *       (/root/reference/cpp/src/Encoder.H:27, Encoder.cpp:17-102)
 * and beneath the verify call sites that compare a chunk's hash with the
 * flood-file string
 *   Flood::_SetupFilesAndChunks      (/root/reference/cpp/src/Flood.cpp:259-275)
 *   ChunkMethodHandler::_HandleRequestChunk (/root/reference/cpp/src/ChunkMethods.cpp:116-123)
 *   ChunkMethodHandler::_HandleSendChunk    (/root/reference/cpp/src/ChunkMethods.cpp:165-167)
 * The C++ wrappers with the reference's exact signatures live in
 * include/libBitFlood/ (libbitflood.so); they call only what is declared here.
 *
 * Conventions (C convention, unlike the reference's ErrorCode where 1 = ok):
 *   - every int-returning call returns LBF_OK (0) on success or a negative
 *     lbf_status; lbf_last_error() returns a thread-local message;
 *   - the caller owns every host array; a context owns device memory,
 *     streams and pinned staging;
 *   - digests are raw 20-byte SHA-1 (big-endian word order, as the reference's
 *     HashFilter emits them, iterhash.h:117-118); chunk i's digest is at
 *     out_digests + 20*i;
 *   - nothing is thrown across the ABI.
 */
#ifndef LBF_HASH_H_
#define LBF_HASH_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LBF_ABI_VERSION 1
#define LBF_DIGEST_BYTES 20
#define LBF_B64_CHARS 27

typedef enum lbf_status {
  LBF_OK = 0,
  LBF_ERR_INVALID = -1,   /* bad argument (null pointer, size overflow, ...) */
  LBF_ERR_NO_DEVICE = -2, /* no MI355X visible: the path has no CPU fallback */
  LBF_ERR_HIP = -3,       /* HIP runtime or kernel launch failure */
  LBF_ERR_NOMEM = -4,     /* device or pinned host allocation failed */
  LBF_ERR_IO = -5         /* file could not be opened / read */
} lbf_status;

/* `flags` for the batch calls: where `base`, `offsets`, `sizes`, `expected`
 * and the outputs live. */
#define LBF_HOST_PTR 0
#define LBF_DEVICE_PTR 1

typedef struct lbf_ctx lbf_ctx;

/* ---- library / context ------------------------------------------------- */
int lbf_abi_version(void);
const char* lbf_last_error(void);
/* Number of visible GPUs (0 when none; never an error on a CPU-only host). */
int lbf_device_count(int* out_count);
/* device_mask bit d selects device d; 0 selects every visible device.
 * Fails with LBF_ERR_NO_DEVICE when no GPU is visible.  Host-path staging,
 * read at creation: batches of up to LBF_SLOT_MB MiB (default 512) in HBM
 * device slots (as many as one chain's duration at PCIe rate needs, within
 * LBF_DEVICE_STAGING_MB, default 16384), fed through LBF_SLOTS pinned host
 * slots per worker (2..8, default 3) of up to LBF_PIN_MB MiB (default 128),
 * all grown on demand; LBF_COPY_THREADS host copy threads (default 8).  Pinned staging is allocated on the GPU's NUMA node and
 * the copy threads run on that node's CPUs (LBF_NUMA=0 turns this off). */
int lbf_ctx_create(uint32_t device_mask, lbf_ctx** out_ctx);
void lbf_ctx_destroy(lbf_ctx* ctx);
int lbf_ctx_num_devices(const lbf_ctx* ctx);
/* Host-path workers: one per selected device (LBF_WORKERS_PER_DEVICE=k, a
 * test knob read at creation, gives k per device).  A batch is split into
 * contiguous index ranges, one per worker, each on its own host thread. */
int lbf_ctx_num_workers(const lbf_ctx* ctx);
/* Placement of worker `worker` (diagnostics): its device, that device's NUMA
 * node (-1 unknown or LBF_NUMA=0), the NUMA node holding its pinned staging
 * (-1 unknown), and how many CPUs its host threads are bound to (0 unbound).
 * Any output pointer may be NULL. */
int lbf_ctx_worker_info(const lbf_ctx* ctx, int worker, int* device, int* numa_node, int* staging_node,
                        int* bound_cpus);

/* ---- batched chunk hashing (Encoder::EncodeFile's per-chunk hash) --------
 * Chunk i is the byte range [offsets[i], offsets[i] + sizes[i]) of `base`.
 * LBF_HOST_PTR: base/offsets/sizes/out are host memory; `base_len` bounds
 *   the readable range of `base`.  Chunks are streamed through pinned staging
 *   to the context's devices (contiguous index ranges per device).
 * LBF_DEVICE_PTR: everything is device memory of the context's first device
 *   and the call is synchronous on the context stream. */
int lbf_sha1_batch(lbf_ctx* ctx, const uint8_t* base, uint64_t base_len,
                   const uint64_t* offsets, const uint32_t* sizes, uint64_t n,
                   uint8_t* out_digests, int flags);

/* ---- batched verify (Flood.cpp:259-275, ChunkMethods.cpp:116-123,165-167)
 * verdicts[i] = 1 when SHA-1(chunk i) equals expected[20*i .. 20*i+20),
 * else 0.  The comparison happens on the device. */
int lbf_verify_batch(lbf_ctx* ctx, const uint8_t* base, uint64_t base_len,
                     const uint64_t* offsets, const uint32_t* sizes, uint64_t n,
                     const uint8_t* expected, uint8_t* verdicts, int flags);

/* ---- caller-pinned sources ------------------------------------------------
 * Register [ptr, ptr + len) of caller host memory with the context (pinned
 * for all of its devices; whole pages).  A LBF_HOST_PTR batch whose
 * [base, base + base_len) lies in a registered range is copied to the device
 * straight from it, one H2D per run of adjacent chunks, instead of passing
 * through the context's pinned staging: host DRAM then carries each byte
 * once, not three times (the staging memcpy's read and write, then the DMA
 * read).  Groups of small scattered chunks (runs under 1 MiB on average)
 * still go through staging.  On one MI355X the direct route ran 14 against
 * 12 GiB/s at 64 MiB and 50 against 34-50 GiB/s at 4 GiB.
 * Meant for buffers reused across calls (a peer's receive arenas, a resident
 * file image): the first registration of pages costs about as much as one
 * staged pass over them -- 4 GiB of touched 4 KiB pages 168-233 ms (what new[]
 * and malloc give), 7.5 ms on transparent huge pages, ~700 ms on pages never
 * touched (the registration faults them in) -- and that cost lands in this
 * call, not in the first direct copy; registering pages HIP registered before
 * in the process is cheap, unregistering ~0.03 ms (tools/register_cost.py,
 * profiles/r06/register_cost/).  A call that overlaps pages a running job
 * pinned on the fly (LBF_AUTOPIN=1) waits for
 * that job to end, then pins the range itself.  Memory
 * that is already pinned is accepted and left pinned.  Pinning is per page:
 * ranges held by one context may not share a page (give each registered
 * buffer pages of its own).  Unregister (with the pointer passed here) before
 * freeing the memory; lbf_ctx_destroy unregisters what is left. */
int lbf_host_register(lbf_ctx* ctx, const void* ptr, uint64_t len);
int lbf_host_unregister(lbf_ctx* ctx, const void* ptr);
/* Cumulative chunk bytes this context's host-pointer and file batches sent
 * through its pinned staging and straight from registered memory
 * (diagnostics; either pointer may be NULL). */
int lbf_ctx_staging_stats(lbf_ctx* ctx, uint64_t* staged_bytes, uint64_t* direct_bytes);

/* ---- chunks read straight from a file ------------------------------------
 * Chunk i = bytes [offsets[i], offsets[i] + sizes[i]) of the file at `path`,
 * read with pread into the context's pinned staging (no intermediate copy),
 * overlapped with H2D copies and kernels.  This is EncodeFile's fread loop
 * (Encoder.cpp:54-72) and _SetupFilesAndChunks' fseek/fread loop
 * (Flood.cpp:259-275) batched.
 * expected == NULL: hash mode, `out` receives n*20 digest bytes; a chunk that
 *   cannot be read in full fails the call with LBF_ERR_IO.
 * expected != NULL: verify mode, `out` receives n verdict bytes; a chunk that
 *   cannot be read in full (missing file, past EOF) gets verdict 0, as the
 *   reference leaves such chunks '0'. */
int lbf_file_ranges(lbf_ctx* ctx, const char* path, const uint64_t* offsets, const uint32_t* sizes,
                    uint64_t n, const uint8_t* expected, uint8_t* out);
/* The same over several files in ONE pipelined batch: chunk i is bytes
 * [offsets[i], offsets[i] + sizes[i]) of paths[file_of[i]] (file_of may be
 * NULL when n_files == 1).  This is EncodeFile's loop over m_files
 * (Encoder.cpp:40-79) and _SetupFilesAndChunks' loop over the flood's files
 * (Flood.cpp:239-287) as one call: every chunk's serial SHA-1 chain costs the
 * same whatever the batch, so per-file calls pay it once per file.  Per-chunk
 * semantics as lbf_file_ranges; a file that cannot be opened fails hash mode
 * with LBF_ERR_IO and gives verdict 0 to all its chunks in verify mode. */
int lbf_files_ranges(lbf_ctx* ctx, const char* const* paths, uint32_t n_files, const uint32_t* file_of,
                     const uint64_t* offsets, const uint32_t* sizes, uint64_t n, const uint8_t* expected,
                     uint8_t* out);

/* ---- received chunks as base64 text (ChunkMethods.cpp:137-167) -----------
 * The receiver's two per-chunk passes on the device: XML-RPC's base64 decode
 * of the SendChunk payload (XmlRpcValue.cpp:417-436, xmlrpc++ 0.7
 * base64.h:215-330) and the verify.  Chunk i arrived as the base64 text
 * text[text_offsets[i], + text_lens[i]) (host memory; the bytes between
 * `<base64>` and `</base64>`).  It is decoded with xmlrpc++'s rules --
 * characters outside the alphabet are skipped; the first group of four that
 * holds '=' ends the data ("xx==" one byte, "xxx=" two); an incomplete last
 * group is dropped -- and verdicts[i] = 1 when the decoded length equals
 * expected_sizes[i] (ChunkMethods.cpp:156) and its SHA-1 equals
 * expected[20*i .. 20*i+20).  out_sizes[i] (may be NULL) receives the decoded
 * length, or expected_sizes[i] + 1 when the text decodes to more.  With `out`
 * non-NULL the decoded bytes land at out[out_offsets[i], + expected_sizes[i])
 * (host memory); the bytes of a slot past its decoded length are zeroed,
 * and no byte of `out` outside the slots is written.  Overlapping slots are
 * refused (LBF_ERR_INVALID).  Synchronous, on the context's first device.
 * Text and output in memory registered with lbf_host_register move by DMA
 * without staging.  lbf_ctx_b64_stats counts the chunks whose text had the
 * encoder's own layout (decoded in one pass) and the others (decoded by the
 * general two-pass kernel).  A chunk of more than 1 GiB (expected_sizes) or
 * 1.5 GiB of text is refused (LBF_ERR_INVALID): the kernels keep positions
 * within a chunk in 32 bits. */
int lbf_b64_verify_batch(lbf_ctx* ctx, const char* text, uint64_t text_len, const uint64_t* text_offsets,
                         const uint32_t* text_lens, uint64_t n, const uint32_t* expected_sizes,
                         const uint8_t* expected, uint8_t* out, uint64_t out_len, const uint64_t* out_offsets,
                         uint32_t* out_sizes, uint8_t* verdicts);

/* ---- chunks to send, encoded as base64 text (ChunkMethods.cpp:89-135) ----
 * The sender's per-chunk passes on the device: the seeder's re-verify
 * (ChunkMethods.cpp:116-123) and XML-RPC's base64 encode of the SendChunk
 * payload (XmlRpcValue::binaryToXml, xmlrpc++ 0.7 base64.h:154-210), from one
 * device copy of the bytes.  Chunk i = data[offsets[i], + sizes[i]) (host
 * memory): verdicts[i] = 1 when its SHA-1 equals expected[20*i .. 20*i+20);
 * its text -- four characters per three bytes, a space (the frame's newline)
 * after every 18th complete group, "xx==" / "xxx=" for a last one or two
 * bytes -- lands at text[text_offsets[i], + lbf_b64_put_length(sizes[i]))
 * whatever the verdict; no byte of `text` outside the slots is written, and
 * overlapping slots are refused (LBF_ERR_INVALID), and so is a chunk of more
 * than 1 GiB.  Synchronous, on the context's first device. */
int lbf_verify_encode_b64_batch(lbf_ctx* ctx, const uint8_t* data, uint64_t data_len, const uint64_t* offsets,
                                const uint32_t* sizes, uint64_t n, const uint8_t* expected, uint8_t* verdicts,
                                char* text, uint64_t text_len, const uint64_t* text_offsets);
/* Chunks of lbf_b64_verify_batch calls on this context so far, by decode
 * path (diagnostics; either pointer may be NULL). */
int lbf_ctx_b64_stats(lbf_ctx* ctx, uint64_t* one_pass_chunks, uint64_t* general_chunks);
/* Length of that text for a chunk of `size` bytes (xmlrpc++'s encoder). */
uint64_t lbf_b64_put_length(uint64_t size);

/* ---- single buffer (Encoder::Base64Encode's hash, host memory) ---------- */
int lbf_sha1_one(lbf_ctx* ctx, const uint8_t* data, uint32_t size, uint8_t out_digest[20]);

/* ---- digest <-> 27-char string (basecode.cpp:39-104, Encoder.cpp:104-105)
 * lbf_b64_27 writes 27 chars + NUL.  lbf_b64_27_decode accepts exactly 27
 * chars of the standard alphabet whose last char carries 4 data bits and 2
 * zero bits; anything else returns LBF_ERR_INVALID. */
void lbf_b64_27(const uint8_t digest[20], char out[28]);
int lbf_b64_27_decode(const char* in, size_t len, uint8_t out_digest[20]);

/* ---- device-resident asynchronous entry points ---------------------------
 * All pointers are device memory on the current HIP device; `stream` is a
 * hipStream_t (NULL = the default stream).  These enqueue and return; they
 * are what bench.py times and what the pipelined host paths use.
 * d_expected/d_verdicts may be NULL (hash only); d_digests may be NULL when
 * only verdicts are wanted. */
int lbf_sha1_launch(const uint8_t* d_base, const uint64_t* d_offsets,
                    const uint32_t* d_sizes, uint64_t n, uint8_t* d_digests,
                    const uint8_t* d_expected, uint8_t* d_verdicts, void* stream);
/* Uniform chunking of one region (one file laid out contiguously):
 * chunk i = [i*chunk_size, min((i+1)*chunk_size, len)), i in [first, first+n). */
int lbf_sha1_uniform_launch(const uint8_t* d_base, uint64_t len, uint32_t chunk_size,
                            uint64_t first_chunk, uint64_t n, uint8_t* d_digests,
                            const uint8_t* d_expected, uint8_t* d_verdicts, void* stream);
/* Kernel variant selection for the two launchers above (0 = automatic):
 * shipped are 1 lane, 7 pc4 (schedule read as 8-byte pairs), 10 pcx5,
 * 11 lds2 and 12 pc4x2; the superseded and diagnostic variants exist only in
 * the A/B library of tools/experimental/, and the shipped library rejects
 * them with LBF_ERR_INVALID.  Exposed for benchmarking and tests; see
 * DESIGN.md "kernels".  lbf_kernel_for(n) is the variant a launch of n
 * chunks runs under the current setting. */
int lbf_set_kernel_variant(int variant);
int lbf_get_kernel_variant(void);
int lbf_kernel_for(uint64_t n_chunks);

/* Synthetic bytes (counter-mode splitmix64): fill
 * d_buf[0..len) with stream `seed` starting at stream byte `start`
 * (start % 8 == 0, d_buf 16-byte aligned). */
int lbf_fill_synthetic(uint8_t* d_buf, uint64_t len, uint64_t seed, uint64_t start, void* stream);

/* Tiny device-memory helpers so C/ctypes callers need no HIP headers. */
int lbf_dev_malloc(void** out_ptr, uint64_t bytes);
int lbf_dev_free(void* ptr);
int lbf_memcpy_h2d(void* dst, const void* src, uint64_t bytes);
int lbf_memcpy_d2h(void* dst, const void* src, uint64_t bytes);
int lbf_set_device(int device);
int lbf_device_synchronize(void);
int lbf_stream_create(void** out_stream);
int lbf_stream_destroy(void* stream);
int lbf_stream_synchronize(void* stream);
/* Time `reps` back-to-back launches of lbf_sha1_uniform_launch on `stream`
 * with HIP events recorded on that stream; writes the mean ms per launch. */
int lbf_time_uniform(const uint8_t* d_base, uint64_t len, uint32_t chunk_size,
                     uint64_t first_chunk, uint64_t n, uint8_t* d_digests, int reps,
                     void* stream, float* out_ms_per_launch);

#ifdef __cplusplus
}
#endif

#endif /* LBF_HASH_H_ */
