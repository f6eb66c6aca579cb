// FloodFile.cpp -- flood-file XML writer/reader without Xerces.
//
// Writer: reproduces what the reference gets from Xerces-C 2.6.0's DOMWriter
// with fgDOMWRTFormatPrettyPrint on the element tree FloodFile::ToXML builds
// (/root/reference/cpp/src/FloodFile.cpp:42-142), serialised with
// writeToString(*rootElem):
//   - each element starts on a new line (DOMWriterImpl.cpp:970-981), preceded
//     by one extra blank line when it sits at level 1 (:971-972);
//   - two spaces of indent per level (printIndent, :1773-1788);
//   - childless elements close with "/>" (:1198-1210); otherwise the end tag
//     goes on its own line, with one extra blank line at level 0 (:1171-1191);
//   - attributes in name order: DOMAttrMapImpl keeps its node list sorted
//     (binary search findNamePoint, DOMAttrMapImpl.cpp:111-150);
//   - attribute values escape & < " and LF (XMLFormatter.cpp:78-84), LF as
//     the hex char ref "&#xA;" (writeCharRef, XMLFormatter.cpp:562-581);
//   - line end LF (gEOLSeq, DOMWriterImpl.cpp:261-264,773).
// Reader: the subset FromXML relies on (FloodFile.cpp:156-322) -- elements
// and attributes, entity and char refs, comments/PIs skipped, any whitespace.
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <string.h>
#include <sys/socket.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <fstream>
#include <sstream>

#include "libBitFlood/Encoder.H"
#include "libBitFlood/FloodFile.H"

namespace libBitFlood {

namespace {

std::atomic<bool> g_resolve_hosts{true};

const char* kRoot = "BitFlood";
const char* kFileInfo = "FileInfo";
const char* kFile = "File";
const char* kChunk = "Chunk";
const char* kTracker = "Tracker";

void escape_attr(std::string& out, const std::string& v) {
  for (char ch : v) {
    switch (ch) {
      case '&': out += "&amp;"; break;
      case '<': out += "&lt;"; break;
      case '"': out += "&quot;"; break;
      case '\n': out += "&#xA;"; break;
      default: out += ch;
    }
  }
}

void attr(std::string& out, const char* name, const std::string& value) {
  out += ' ';
  out += name;
  out += "=\"";
  escape_attr(out, value);
  out += '"';
}

// ---- minimal XML reader ----------------------------------------------------
struct Node {
  std::string name;
  std::vector<std::pair<std::string, std::string>> attrs;
  std::vector<Node> kids;
  const std::string* get(const char* key) const {
    for (const auto& a : attrs)
      if (a.first == key) return &a.second;
    return nullptr;
  }
};

struct Parser {
  const std::string& s;
  size_t p = 0;
  bool ok = true;
  explicit Parser(const std::string& src) : s(src) {}

  static bool is_space(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n'; }
  void skip_ws() { while (p < s.size() && is_space(s[p])) ++p; }
  bool starts(const char* lit) const { return s.compare(p, strlen(lit), lit) == 0; }

  void skip_misc() {  // whitespace, text, comments, PIs, DOCTYPE between elements
    for (;;) {
      while (p < s.size() && s[p] != '<') ++p;
      if (p >= s.size()) return;
      if (starts("<!--")) {
        size_t e = s.find("-->", p + 4);
        p = e == std::string::npos ? s.size() : e + 3;
      } else if (starts("<?") || starts("<!")) {
        size_t e = s.find('>', p + 2);
        p = e == std::string::npos ? s.size() : e + 1;
      } else {
        return;
      }
    }
  }

  // An attribute value as an XML 1.0 parser reports it (§3.3.3, what Xerces
  // hands FloodFile.cpp:74): line ends normalised (CR LF or a lone CR is one
  // LF, §2.11), every literal TAB, LF or CR then a space, entity and character
  // references replaced (a reference to TAB, LF or CR keeps that character).
  static bool decode(const std::string& raw, std::string& out) {
    out.clear();
    for (size_t i = 0; i < raw.size(); ++i) {
      if (raw[i] == '\r' || raw[i] == '\n' || raw[i] == '\t') {
        if (raw[i] == '\r' && i + 1 < raw.size() && raw[i + 1] == '\n') ++i;
        out += ' ';
        continue;
      }
      if (raw[i] != '&') {
        out += raw[i];
        continue;
      }
      const size_t semi = raw.find(';', i);
      if (semi == std::string::npos) return false;
      const std::string ent = raw.substr(i + 1, semi - i - 1);
      if (ent == "amp") out += '&';
      else if (ent == "lt") out += '<';
      else if (ent == "gt") out += '>';
      else if (ent == "quot") out += '"';
      else if (ent == "apos") out += '\'';
      else if (!ent.empty() && ent[0] == '#') {
        const bool hex = ent.size() > 1 && (ent[1] == 'x' || ent[1] == 'X');
        const char* digits = ent.c_str() + (hex ? 2 : 1);
        char* end = nullptr;
        const unsigned long cp = strtoul(digits, &end, hex ? 16 : 10);
        // a character reference names one XML Char (XML 1.0 §2.2): not empty,
        // no trailing junk, no surrogate, nothing past U+10FFFF
        if (end == digits || *end != '\0' || cp == 0 || cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF)) return false;
        if (cp < 0x80) {  // UTF-8, one to four bytes
          out += (char)cp;
        } else if (cp < 0x800) {
          out += (char)(0xC0 | (cp >> 6));
          out += (char)(0x80 | (cp & 0x3F));
        } else if (cp < 0x10000) {
          out += (char)(0xE0 | (cp >> 12));
          out += (char)(0x80 | ((cp >> 6) & 0x3F));
          out += (char)(0x80 | (cp & 0x3F));
        } else {  // round 6: characters past the BMP took three bytes and lost their top bits
          out += (char)(0xF0 | (cp >> 18));
          out += (char)(0x80 | ((cp >> 12) & 0x3F));
          out += (char)(0x80 | ((cp >> 6) & 0x3F));
          out += (char)(0x80 | (cp & 0x3F));
        }
      } else {
        return false;
      }
      i = semi;
    }
    return true;
  }

  bool element(Node& n) {
    if (p >= s.size() || s[p] != '<') return false;
    ++p;
    size_t b = p;
    while (p < s.size() && !is_space(s[p]) && s[p] != '>' && s[p] != '/') ++p;
    n.name = s.substr(b, p - b);
    for (;;) {
      skip_ws();
      if (p >= s.size()) return false;
      if (s[p] == '/') {
        if (p + 1 < s.size() && s[p + 1] == '>') {
          p += 2;
          return true;
        }
        return false;
      }
      if (s[p] == '>') {
        ++p;
        break;
      }
      b = p;
      while (p < s.size() && s[p] != '=' && !is_space(s[p])) ++p;
      std::string key = s.substr(b, p - b);
      skip_ws();
      if (p >= s.size() || s[p] != '=') return false;
      ++p;
      skip_ws();
      if (p >= s.size() || (s[p] != '"' && s[p] != '\'')) return false;
      const char q = s[p++];
      b = p;
      while (p < s.size() && s[p] != q) ++p;
      if (p >= s.size()) return false;
      std::string val;
      if (!decode(s.substr(b, p - b), val)) return false;
      ++p;
      n.attrs.emplace_back(std::move(key), std::move(val));
    }
    // children until the matching end tag
    for (;;) {
      skip_misc();
      if (p >= s.size()) return false;
      if (starts("</")) {
        const size_t e = s.find('>', p);
        if (e == std::string::npos) return false;
        std::string nm = s.substr(p + 2, e - p - 2);
        while (!nm.empty() && is_space(nm.back())) nm.pop_back();
        p = e + 1;
        return nm == n.name;
      }
      n.kids.emplace_back();
      if (!element(n.kids.back())) return false;
    }
  }
};

// getElementsByTagName: every descendant with that name, document order.
void collect(const Node& n, const char* name, std::vector<const Node*>& out) {
  for (const Node& k : n.kids) {
    if (k.name == name) out.push_back(&k);
    collect(k, name, out);
  }
}

// U32 attribute as the reference reads it: wstringstream >> U32 (0 on failure)
U32 to_u32(const std::string* v) {
  if (!v) return 0;
  std::istringstream is(*v);
  unsigned long long x = 0;
  if (!(is >> x) || x > 0xFFFFFFFFull) return 0;
  return (U32)x;
}

U64 to_u64(const std::string* v) {
  if (!v) return 0;
  std::istringstream is(*v);
  unsigned long long x = 0;
  if (!(is >> x)) return 0;
  return (U64)x;
}

// gethostbyname + inet_ntoa in the reference (FloodFile.cpp:290-291).
std::string resolve_ipv4(const std::string& host) {
  if (!g_resolve_hosts.load()) return host;
  addrinfo hints{};
  hints.ai_family = AF_INET;
  addrinfo* res = nullptr;
  if (getaddrinfo(host.c_str(), nullptr, &hints, &res) != 0 || !res) return host;
  char buf[INET_ADDRSTRLEN] = {0};
  const sockaddr_in* sin = reinterpret_cast<const sockaddr_in*>(res->ai_addr);
  inet_ntop(AF_INET, &sin->sin_addr, buf, sizeof(buf));
  freeaddrinfo(res);
  return buf[0] ? std::string(buf) : host;
}

bool chunk_less(const FloodFile::Chunk& a, const FloodFile::Chunk& b) { return a.m_index < b.m_index; }

}  // namespace

void FloodFile::SetResolveTrackerHosts(bool i_resolve) { g_resolve_hosts.store(i_resolve); }

Error::ErrorCode FloodFile::ToXML(std::string& o_xml) { return ToXML(o_xml, SizeAttr::RefU32); }

Error::ErrorCode FloodFile::ToXML(std::string& o_xml, SizeAttr i_sizes) {
  std::string x;
  x.reserve(128 + 90 * 1024);
  x += "\n<";  // root element at level 0: one newline, no indent
  x += kRoot;
  x += '>';
  // FileInfo (level 1): blank line, 2-space indent
  x += "\n\n  <";
  x += kFileInfo;
  if (m_files.empty()) {
    x += "/>";
  } else {
    x += '>';
    for (const auto& kv : m_files) {
      const File& f = *kv.second;
      x += "\n    <";
      x += kFile;
      attr(x, "name", f.m_name);
      // RefU32: what the reference's U32 filesize holds after the fread loop
      // (Encoder.cpp:42,59,76) -- the size modulo 2^32
      attr(x, "size", std::to_string(i_sizes == SizeAttr::RefU32 ? (U64)(U32)f.m_size : f.m_size));
      if (f.m_chunks.empty()) {
        x += "/>";
        continue;
      }
      x += '>';
      for (const Chunk& c : f.m_chunks) {
        x += "\n      <";
        x += kChunk;
        attr(x, "hash", c.m_hash);
        attr(x, "index", std::to_string(c.m_index));
        attr(x, "size", std::to_string(c.m_size));
        attr(x, "weight", std::to_string(c.m_weight));
        x += "/>";
      }
      x += "\n    </";
      x += kFile;
      x += '>';
    }
    x += "\n  </";
    x += kFileInfo;
    x += '>';
  }
  for (const TrackerInfo& t : m_trackers) {
    x += "\n\n  <";
    x += kTracker;
    attr(x, "host", t.m_host);
    attr(x, "port", std::to_string(t.m_port));
    x += "/>";
  }
  x += "\n\n</";  // root has children: its end tag after a blank line
  x += kRoot;
  x += '>';
  o_xml.swap(x);
  return Error::NO_ERROR_LBF;
}

Error::ErrorCode FloodFile::FromXML(const std::string& i_xml) {
  Parser ps(i_xml);
  ps.skip_misc();
  Node root;
  const bool parsed = ps.element(root);
  if (parsed) {
    // The reference searches the document; the root element is included in
    // that search only if it matches, which it never does for FileInfo.
    std::vector<const Node*> infos;
    if (root.name == kFileInfo) infos.push_back(&root);
    collect(root, kFileInfo, infos);
    if (infos.size() == 1) {  // FloodFile.cpp:230: exactly one FileInfo
      std::vector<const Node*> files;
      collect(*infos[0], kFile, files);
      for (const Node* fn : files) {
        FileSPtr f(new File());
        const std::string* nm = fn->get("name");
        f->m_name = nm ? *nm : std::string();
        f->m_size = to_u64(fn->get("size"));
        std::vector<const Node*> chunks;
        collect(*fn, kChunk, chunks);
        for (const Node* cn : chunks) {
          Chunk c;
          const std::string* h = cn->get("hash");
          c.m_hash = h ? *h : std::string();
          c.m_index = to_u32(cn->get("index"));
          c.m_weight = to_u32(cn->get("weight"));
          c.m_size = to_u32(cn->get("size"));
          f->m_chunks.push_back(c);
        }
        std::stable_sort(f->m_chunks.begin(), f->m_chunks.end(), chunk_less);  // FloodFile.cpp:268
        // A reference-written (wrapped U32) size of a file >= 4 GiB: the chunk
        // sizes carry the true total, which the size matches modulo 2^32.
        U64 sum = 0;
        for (const Chunk& c : f->m_chunks) sum += c.m_size;
        if (sum > 0xFFFFFFFFull && f->m_size == (sum & 0xFFFFFFFFull)) f->m_size = sum;
        m_files[f->m_name] = f;
      }
    }
    std::vector<const Node*> trackers;
    if (root.name == kTracker) trackers.push_back(&root);
    collect(root, kTracker, trackers);
    for (const Node* tn : trackers) {
      TrackerInfo t;
      const std::string* h = tn->get("host");
      t.m_host = resolve_ipv4(h ? *h : std::string());
      t.m_port = to_u32(tn->get("port"));
      std::ostringstream id;
      id << t.m_host << t.m_port;  // FloodFile.cpp:297-300
      Encoder::Base64Encode(reinterpret_cast<const U8*>(id.str().data()), (U32)id.str().size(), t.m_id);
      m_trackers.push_back(t);
    }
  }
  ComputeHash(m_contentHash);  // FloodFile.cpp:314, also after a failed parse
  // The reference returns NO_ERROR_LBF whatever the parser saw
  // (FloodFile.cpp:321); a malformed document simply yields no files.
  return Error::NO_ERROR_LBF;
}

Error::ErrorCode FloodFile::ComputeHash(std::string& o_hash) {
  std::string tohash;
  for (const auto& kv : m_files) {
    tohash += kv.second->m_name;
    for (const Chunk& c : kv.second->m_chunks) tohash += c.m_hash;
  }
  return Encoder::Base64Encode(reinterpret_cast<const U8*>(tohash.data()), (U32)tohash.size(), o_hash);
}

Error::ErrorCode FloodFile::ToXMLFile(const std::string& i_path, bool i_crlf, SizeAttr i_sizes) {
  std::string xml;
  ToXML(xml, i_sizes);
  if (i_crlf) {
    std::string w;
    w.reserve(xml.size() + xml.size() / 16);
    for (char ch : xml) {
      if (ch == '\n') w += '\r';
      w += ch;
    }
    xml.swap(w);
  }
  FILE* f = fopen(i_path.c_str(), "wb");
  if (!f) return Error::UNKNOWN_ERROR_LBF;
  const bool ok = fwrite(xml.data(), 1, xml.size(), f) == xml.size();
  return (fclose(f) == 0 && ok) ? Error::NO_ERROR_LBF : Error::UNKNOWN_ERROR_LBF;
}

Error::ErrorCode FloodFile::FromXMLFile(const std::string& i_path) {
  std::ifstream in(i_path, std::ios::binary);
  if (!in) return Error::UNKNOWN_ERROR_LBF;
  std::ostringstream ss;
  ss << in.rdbuf();
  return FromXML(ss.str());
}

}  // namespace libBitFlood
