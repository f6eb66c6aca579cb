// lbf_latency.cpp -- latency of the single-buffer entry point
// Encoder::Base64Encode (/root/reference/cpp/src/Encoder.cpp:107-120) on the
// sizes its non-batched callers pass: a peer / tracker id (host + port,
// Peer.cpp:20-26, FloodFile.cpp:297-300: ~20 B), the content hash input of a
// C2 flood file (FloodFile.cpp:324-349: name + 16,384 x 27 chars ≈ 442 KB),
// and single chunks (64 KiB, 256 KiB).  Prints one JSON line: the first call
// (context creation included) and the warm median / p99 per size.
//
//   lbf_latency [--reps N]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "libBitFlood/Encoder.H"

using namespace libBitFlood;
using Clock = std::chrono::steady_clock;

int main(int argc, char** argv) {
  int reps = 200;
  for (int i = 1; i < argc; ++i)
    if (std::string(argv[i]) == "--reps" && i + 1 < argc) reps = atoi(argv[++i]);
  struct Case {
    const char* name;
    size_t size;
  };
  const Case cases[] = {{"peer_id_20B", 20}, {"content_hash_c2_442KB", 5 + 16384 * 27},
                        {"chunk_64KiB", 65536}, {"chunk_256KiB", 262144}};
  std::vector<unsigned char> buf(262144 * 2);
  for (size_t k = 0; k < buf.size(); ++k) buf[k] = (unsigned char)(k * 131 + 7);
  std::string out;
  double first_us = 0;
  {
    auto t0 = Clock::now();
    if (Encoder::Base64Encode(buf.data(), 20, out) != Error::NO_ERROR_LBF) {
      fprintf(stderr, "lbf_latency: %s\n", Encoder::LastError());
      return 2;
    }
    first_us = std::chrono::duration<double, std::micro>(Clock::now() - t0).count();
  }
  printf("{\"first_call_us\": %.1f, \"reps\": %d", first_us, reps);
  for (const Case& c : cases) {
    std::vector<double> us;
    for (int r = 0; r < reps; ++r) {
      auto t0 = Clock::now();
      if (Encoder::Base64Encode(buf.data() + (r % 7), (U32)c.size, out) != Error::NO_ERROR_LBF) return 2;
      us.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
    }
    std::sort(us.begin(), us.end());
    printf(", \"%s\": {\"p50_us\": %.1f, \"p99_us\": %.1f, \"min_us\": %.1f}", c.name, us[us.size() / 2],
           us[std::min(us.size() - 1, us.size() * 99 / 100)], us[0]);
  }
  printf("}\n");
  return 0;
}
