// lbf_verify -- the startup half of /root/reference/cpp/test_client
// (test_client.cpp:47-69 -> ParseFloodFile :79-119 -> Flood::Initialize ->
// _SetupFilesAndChunks): read a flood file and re-verify every chunk already
// on disk, batched on the GPU.  Prints one line per file:
//   <name> <chunks> <verified> <chunkmap>
// and the flood's content hash.
//   lbf_verify <flood> [--root DIR] [--no-resolve] [--devices MASK]
#include <cstdlib>
#include <iostream>
#include <string>

#include "libBitFlood/Encoder.H"
#include "libBitFlood/Flood.H"

using namespace libBitFlood;

int main(int argc, char* argv[]) {
  std::string flood, root;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "--root" && i + 1 < argc) root = argv[++i];
    else if (a == "--no-resolve") FloodFile::SetResolveTrackerHosts(false);
    else if (a == "--devices" && i + 1 < argc) Encoder::SetDeviceMask((U32)strtoul(argv[++i], nullptr, 0));
    else flood = a;
  }
  if (flood.empty()) {
    std::cerr << "usage: lbf_verify <flood> [--root DIR] [--no-resolve]" << std::endl;
    return 1;
  }
  FloodFileSPtr ff(new FloodFile());
  if (ff->FromXMLFile(flood) != Error::NO_ERROR_LBF) {
    std::cerr << "cannot read " << flood << std::endl;
    return 2;
  }
  Flood f;
  f.m_rootdir = root;
  if (f.Initialize(ff) != Error::NO_ERROR_LBF) {
    std::cerr << "verify failed: " << Encoder::LastError() << std::endl;
    return 3;
  }
  for (const auto& kv : f.m_runtimefiles) {
    size_t ok = 0;
    for (char c : kv.second.m_chunkmap) ok += c == '1';
    std::cout << kv.first << " " << kv.second.m_chunkmap.size() << " " << ok << " " << kv.second.m_chunkmap << "\n";
  }
  std::cout << "content_hash " << ff->m_contentHash << "\n";
  std::cout << "to_download " << f.m_chunkstodownload.size() << std::endl;
  return 0;
}
