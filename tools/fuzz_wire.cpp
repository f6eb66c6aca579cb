// tools/fuzz_wire.cpp -- diagnostic (not product code): random and mutated
// inputs through the peer-frame parser, the base64 decoder and the flood-file
// reader, for an ASAN/UBSan build on the host:
//   g++ -O1 -g -std=c++17 -fsanitize=address,undefined -I../include fuzz_wire.cpp \
//     ../bitflood_amd/host/{PeerWire,FloodFile,Encoder,Flood}.cpp -L../bitflood_amd/lib -llbfhash -o build/fuzz_wire
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "libBitFlood/FloodFile.H"
#include "libBitFlood/PeerWire.H"

using namespace libBitFlood;

int main(int argc, char** argv) {
  const long iters = argc > 1 ? atol(argv[1]) : 200000;
  std::mt19937_64 rng(12345);
  std::vector<U8> chunk(3000);
  for (auto& b : chunk) b = (U8)rng();
  const std::string seeds[] = {
      PeerWire::EncodeSendChunk("a&b.bin", 7, chunk.data(), (U32)chunk.size()),
      PeerWire::EncodeMethod(PeerWire::kRequestChunk, {PeerWire::Value::Str("x"), PeerWire::Value::Int(3)}),
      "<?xml version=\"1.0\"?>\n<BitFlood><FileInfo><File name=\"a\" size=\"5\"><Chunk hash=\"qZk+NkcGgWq6PiVxeFDCbJzQ2J0\""
      " index=\"0\" size=\"5\" weight=\"0\"/></File></FileInfo><Tracker host=\"h\" port=\"1\"/></BitFlood>",
  };
  const char alphabet[] = "<>/&;=\"' \n\r\t+ABCDabcd0123paramvluebs64i4methodNamFileChunkTrackerindexsizehash";
  long checks = 0;
  for (long it = 0; it < iters; ++it) {
    std::string s = seeds[rng() % 3];
    const int muts = 1 + (int)(rng() % 8);
    for (int m = 0; m < muts && !s.empty(); ++m) {
      const size_t pos = rng() % s.size();
      switch (rng() % 4) {
        case 0: s[pos] = alphabet[rng() % (sizeof(alphabet) - 1)]; break;
        case 1: s.erase(pos, 1 + rng() % 16); break;
        case 2: s.insert(pos, std::string(1 + rng() % 8, alphabet[rng() % (sizeof(alphabet) - 1)])); break;
        case 3: s.resize(pos); break;
      }
    }
    if (rng() % 16 == 0) {  // pure noise
      s.resize(rng() % 512);
      for (auto& c : s) c = (char)rng();
    }
    std::string method;
    std::vector<PeerWire::Value> params;
    PeerWire::DecodeMethod(s, method, params);
    std::string fname;
    U32 idx = 0;
    size_t n = 0;
    std::vector<U8> out(4096);
    // (ptr, len) APIs get an exact-size heap copy with no terminator, so ASAN
    // sees any read past `len` (a std::string's data() is NUL-terminated).
    std::unique_ptr<char[]> raw(new char[s.size()]);
    if (!s.empty()) memcpy(raw.get(), s.data(), s.size());
    if (PeerWire::DecodeSendChunk(raw.get(), s.size(), fname, idx, out.data(), out.size(), n)) checks += n <= out.size();
    std::vector<U8> small(7);
    PeerWire::Base64Get(raw.get(), s.size(), small.data(), small.size());
    FloodFile f;
    f.FromXML(s);
    ++checks;
  }
  std::printf("fuzz_wire OK %ld iterations (%ld)\n", iters, checks);
  return 0;
}
