// host_tests.cpp -- CPU-only unit tests of the flood-file format (no GPU, no
// hashing): ToXML bytes against the Xerces pretty-print rules traced in
// FloodFile.cpp, FromXML round trips, escapes, CRLF input, chunk ordering.
// Run by tests/test_host_cpp.py (not marked gpu).
#include <cstdio>
#include <cstdlib>
#include <string>

#include "libBitFlood/FloodFile.H"

using namespace libBitFlood;

static int g_fail = 0;
#define CHECK(cond)                                                       \
  do {                                                                    \
    if (!(cond)) {                                                        \
      std::fprintf(stderr, "%s:%d CHECK failed: %s\n", __FILE__, __LINE__, #cond); \
      ++g_fail;                                                           \
    }                                                                     \
  } while (0)

static FloodFile model() {
  FloodFile f;
  FloodFile::FileSPtr a(new FloodFile::File());
  a->m_name = "a.bin";
  a->m_size = 70000;
  FloodFile::Chunk c0{"LgAPp+hXWcf0wlTU2cM+9IHkWac", 0, 65536, 0};
  FloodFile::Chunk c1{"qZk+NkcGgWq6PiVxeFDCbJzQ2J0", 1, 4464, 0};
  a->m_chunks = {c0, c1};
  FloodFile::FileSPtr b(new FloodFile::File());
  b->m_name = "b&c\"<d>\n.bin";
  b->m_size = 0;
  f.m_files[a->m_name] = a;
  f.m_files[b->m_name] = b;
  FloodFile::TrackerInfo t;
  t.m_host = "127.0.0.1";
  t.m_port = 10101;
  f.m_trackers.push_back(t);
  return f;
}

static const char* kExpected =
    "\n<BitFlood>"
    "\n\n  <FileInfo>"
    "\n    <File name=\"a.bin\" size=\"70000\">"
    "\n      <Chunk hash=\"LgAPp+hXWcf0wlTU2cM+9IHkWac\" index=\"0\" size=\"65536\" weight=\"0\"/>"
    "\n      <Chunk hash=\"qZk+NkcGgWq6PiVxeFDCbJzQ2J0\" index=\"1\" size=\"4464\" weight=\"0\"/>"
    "\n    </File>"
    "\n    <File name=\"b&amp;c&quot;&lt;d>&#xA;.bin\" size=\"0\"/>"
    "\n  </FileInfo>"
    "\n\n  <Tracker host=\"127.0.0.1\" port=\"10101\"/>"
    "\n\n</BitFlood>";

int main() {
  FloodFile::SetResolveTrackerHosts(false);
  // 1. writer bytes
  FloodFile m = model();
  std::string xml;
  CHECK(m.ToXML(xml) == Error::NO_ERROR_LBF);
  CHECK(xml == kExpected);
  if (xml != kExpected) std::fprintf(stderr, "got:\n[%s]\n", xml.c_str());

  // 2. empty flood: FileInfo without children closes with "/>"
  FloodFile e;
  std::string ex;
  e.ToXML(ex);
  CHECK(ex == "\n<BitFlood>\n\n  <FileInfo/>\n\n</BitFlood>");

  // 3. reader round trip (LF and CRLF), escapes decoded
  for (int crlf = 0; crlf < 2; ++crlf) {
    std::string src = xml;
    if (crlf) {
      std::string w;
      for (char ch : src) {
        if (ch == '\n') w += '\r';
        w += ch;
      }
      src = w;
    }
    FloodFile r;
    CHECK(r.FromXML(src) == Error::NO_ERROR_LBF);
    CHECK(r.m_files.size() == 2);
    CHECK(r.m_files.count("a.bin") == 1);
    CHECK(r.m_files.count("b&c\"<d>\n.bin") == 1);
    if (r.m_files.count("a.bin")) {
      const FloodFile::File& a = *r.m_files["a.bin"];
      CHECK(a.m_size == 70000);
      CHECK(a.m_chunks.size() == 2);
      CHECK(a.m_chunks[1].m_hash == "qZk+NkcGgWq6PiVxeFDCbJzQ2J0");
      CHECK(a.m_chunks[1].m_size == 4464);
    }
    CHECK(r.m_trackers.size() == 1 && r.m_trackers[0].m_host == "127.0.0.1" && r.m_trackers[0].m_port == 10101);
    std::string again;
    r.ToXML(again);
    CHECK(again == xml);
  }

  // 4. chunks come back sorted by index (FloodFile.cpp:268)
  {
    FloodFile r;
    r.FromXML("<BitFlood><FileInfo><File name=\"x\" size=\"3\">"
              "<Chunk hash=\"h2\" index=\"2\" size=\"1\" weight=\"0\"/>"
              "<Chunk hash=\"h0\" index=\"0\" size=\"1\" weight=\"0\"/>"
              "<Chunk hash=\"h1\" index=\"1\" size=\"1\" weight=\"5\"/>"
              "</File></FileInfo></BitFlood>");
    CHECK(r.m_files.size() == 1);
    if (r.m_files.size() == 1) {
      const FloodFile::V_Chunk& c = r.m_files["x"]->m_chunks;
      CHECK(c.size() == 3 && c[0].m_hash == "h0" && c[1].m_hash == "h1" && c[2].m_hash == "h2");
      CHECK(c[1].m_weight == 5);
    }
  }

  // 5. two FileInfo elements: the reference takes none (FloodFile.cpp:230)
  {
    FloodFile r;
    r.FromXML("<BitFlood><FileInfo><File name=\"x\" size=\"1\"/></FileInfo><FileInfo/></BitFlood>");
    CHECK(r.m_files.empty());
  }

  // 6. 64-bit file sizes are written in full (the reference's U32 wraps)
  {
    FloodFile f;
    FloodFile::FileSPtr big(new FloodFile::File());
    big->m_name = "big";
    big->m_size = 4ull << 30;
    f.m_files["big"] = big;
    std::string x;
    f.ToXML(x);
    CHECK(x.find("size=\"4294967296\"/>") != std::string::npos);
  }

  // 7. malformed input: no crash, no files
  {
    FloodFile r;
    r.FromXML("<BitFlood><FileInfo><File name=\"x\" size=\"1\">");
    CHECK(r.m_files.empty());
    FloodFile r2;
    r2.FromXML("");
    CHECK(r2.m_files.empty());
  }

  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("host_tests OK\n");
  return 0;
}
