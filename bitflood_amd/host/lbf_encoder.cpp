// lbf_encoder -- Linux port of /root/reference/cpp/test_encoder/src/test_encoder.cpp
// (:16-75): encode files into a flood file.
//   lbf_encoder <file> [<file>...] http://host:port/ <out.flood> [--chunksize N] [--crlf] [--devices MASK] [--time]
// With one file: the reference's three positional arguments and the same
// tracker-URL parsing (:44-52).  More files before the URL fill
// ToEncode::m_files in order (Encoder.H:17-25; the reference CLI passes one,
// EncodeFile takes any number -- config C3 is 64 of them).  The chunk size the
// reference hard-wires to 262144 (:56) becomes a flag (config C1 needs 64 KiB).
// --crlf writes the CRLF line ends test_encoder's fopen(..., "w") produces on
// Win32.  --time prints one JSON line: bytes, files, EncodeFile and XML seconds.
// File sizes: the reference's wrapped U32 by default (--ref-u32-size, the
// bytes its encoder writes for a file >= 4 GiB); --true-size writes 64-bit
// sizes instead (FloodFile.H, SizeAttr).
#include <sys/stat.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <sstream>
#include <string>

#include "libBitFlood/Encoder.H"
#include "libBitFlood/FloodFile.H"

using namespace libBitFlood;

int main(int argc, char* argv[]) {
  std::vector<std::string> pos;
  U32 chunksize = 262144;
  bool crlf = false, timing = false;
  FloodFile::SizeAttr sizes = FloodFile::SizeAttr::RefU32;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "--chunksize" && i + 1 < argc) chunksize = (U32)strtoul(argv[++i], nullptr, 10);
    else if (a == "--crlf") crlf = true;
    else if (a == "--time") timing = true;
    else if (a == "--ref-u32-size") sizes = FloodFile::SizeAttr::RefU32;
    else if (a == "--true-size") sizes = FloodFile::SizeAttr::True64;
    else if (a == "--devices" && i + 1 < argc) Encoder::SetDeviceMask((U32)strtoul(argv[++i], nullptr, 0));
    else pos.push_back(a);
  }
  if (pos.size() < 3) {
    std::cerr << "Please use three arguments: the name of the file to encode, the name of the tracker, and the "
                 "name of the flood file"
              << std::endl;
    return 1;
  }
  Encoder::ToEncode::Tracker tracker;
  const std::string url = pos[pos.size() - 2];
  const size_t h_start = url.find("http://") + strlen("http://");
  const size_t p_start = url.find(':', h_start) + 1;
  const size_t u_start = url.find('/', p_start) + 1;
  tracker.first = url.substr(h_start, p_start - h_start - 1);
  std::stringstream port;
  port << url.substr(p_start, u_start - p_start - 1);
  port >> tracker.second;

  Encoder::ToEncode e;
  e.m_files.assign(pos.begin(), pos.end() - 2);
  e.m_chunksize = chunksize;
  e.m_trackers.push_back(tracker);

  using Clock = std::chrono::steady_clock;
  FloodFile out;
  const auto t0 = Clock::now();
  if (Encoder::EncodeFile(e, out) != Error::NO_ERROR_LBF) {
    std::cerr << "EncodeFile failed: " << Encoder::LastError() << std::endl;
    return 2;
  }
  const auto t1 = Clock::now();
  if (out.ToXMLFile(pos.back(), crlf, sizes) != Error::NO_ERROR_LBF) {
    std::cerr << "cannot write " << pos.back() << std::endl;
    return 3;
  }
  const auto t2 = Clock::now();
  if (timing) {
    unsigned long long bytes = 0;
    for (const std::string& f : e.m_files) {
      struct stat st;
      if (stat(f.c_str(), &st) == 0) bytes += (unsigned long long)st.st_size;
    }
    std::printf("{\"files\": %zu, \"bytes\": %llu, \"encode_s\": %.4f, \"xml_s\": %.4f}\n", e.m_files.size(), bytes,
                std::chrono::duration<double>(t1 - t0).count(), std::chrono::duration<double>(t2 - t1).count());
  }
  return 0;
}
