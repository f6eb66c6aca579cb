// PeerWire.cpp -- the reference peer loop's message format (see PeerWire.H for
// the reference files and lines each piece restates).
#include "libBitFlood/PeerWire.H"

#include <ctype.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

namespace libBitFlood {
namespace PeerWire {

const char kRequestChunk[] = "RequestChunk";
const char kSendChunk[] = "SendChunk";
const char kNotifyHaveChunk[] = "NotifyHaveChunk";

namespace {

const char kAlphabet[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
constexpr U8 kEq = 64, kSkip = 255;

struct DecodeTable {
  U8 v[256];
  DecodeTable() {
    memset(v, kSkip, sizeof(v));
    for (int i = 0; i < 64; ++i) v[(U8)kAlphabet[i]] = (U8)i;
    v[(U8)'='] = kEq;
  }
};
const DecodeTable kDecode;

// XmlRpcClient.cpp:14-22 (request framing strings)
const char kRequestBegin[] = "<?xml version=\"1.0\"?>\r\n<methodCall><methodName>";
const char kRequestEndMethodName[] = "</methodName>\r\n";
const char kRequestEnd[] = "</methodCall>\r\n";

void value_xml(const Value& v, std::string& out) {
  switch (v.m_type) {
    case Value::STRING:
      out += "<value>";
      out += XmlEncode(v.m_str);
      out += "</value>";
      break;
    case Value::INT: {
      char buf[32];
      snprintf(buf, sizeof(buf), "%d", v.m_int);
      out += "<value><i4>";
      out += buf;
      out += "</i4></value>";
      break;
    }
    case Value::BINARY:
      out += "<value><base64>";
      Base64Put(v.m_bin.empty() ? nullptr : &v.m_bin[0], v.m_bin.size(), out);
      out += "</base64></value>";
      break;
  }
}

// SendMethod's frame: CR/LF -> ' ', then the '\n' delimiter.
void frame(std::string& s) {
  for (char& c : s)
    if (c == '\n' || c == '\r') c = ' ';
  s += '\n';
}

// XmlRpcUtil::nextTagIs: whitespace, then `tag`.
bool next_tag_is(const char* tag, const char* s, size_t len, size_t& off) {
  size_t p = off;
  while (p < len && isspace((unsigned char)s[p])) ++p;
  const size_t n = strlen(tag);
  if (p + n <= len && memcmp(s + p, tag, n) == 0) {
    off = p + n;
    return true;
  }
  return false;
}

// XmlRpcUtil::getNextTag: the next tag if the next non-space char is '<'.
std::string get_next_tag(const char* s, size_t len, size_t& off) {
  size_t p = off;
  while (p < len && isspace((unsigned char)s[p])) ++p;
  if (p >= len || s[p] != '<') return std::string();
  const size_t b = p;
  while (p < len && s[p] != '>') ++p;
  if (p < len) ++p;
  off = p;
  return std::string(s + b, p - b);
}

const char* find(const char* s, size_t len, size_t from, const char* needle) {
  const size_t n = strlen(needle);
  if (from >= len || n > len - from) return nullptr;
  const char* p = (const char*)memmem(s + from, len - from, needle, n);
  return p;
}

// XmlRpcValue::fromXml for the three value kinds the peer loop sends.  For
// BINARY with `dst` set, decodes into dst instead of v.m_bin.
bool parse_value(const char* s, size_t len, size_t& off, Value& v, U8* dst, size_t cap, size_t* dst_len) {
  const size_t saved = off;
  if (!next_tag_is("<value>", s, len, off)) return false;
  const size_t after_value = off;
  const std::string tag = get_next_tag(s, len, off);
  bool ok = false;
  if (tag == "<i4>" || tag == "<int>") {
    // intFromXml is strtol on the rest of the buffer; the frame is (ptr, len)
    // and need not be NUL-terminated, so strtol runs on a bounded copy.  The
    // leading whitespace strtol skips (any amount) is skipped in the frame
    // first; 63 chars then hold any sign + digits strtol would still accept
    // without saturating differently.
    size_t ws = off;
    while (ws < len && (s[ws] == ' ' || (s[ws] >= '\t' && s[ws] <= '\r'))) ++ws;
    char tok[64];
    const size_t n = std::min(sizeof(tok) - 1, len - ws);
    memcpy(tok, s + ws, n);
    tok[n] = '\0';
    char* end = nullptr;
    const long x = strtol(tok, &end, 10);
    if (end != tok) {
      v.m_type = Value::INT;
      v.m_int = (int)x;
      off = ws + (size_t)(end - tok);
      ok = next_tag_is(tag == "<i4>" ? "</i4>" : "</int>", s, len, off);
    }
  } else if (tag.empty() || tag == "<string>" || tag == "</value>") {
    if (tag == "</value>") off = after_value;  // blank string without <string>
    const char* lt = (const char*)memchr(s + off, '<', len - off);  // stringFromXml
    if (lt) {
      v.m_type = Value::STRING;
      v.m_str = XmlDecode(std::string(s + off, lt));
      off = (size_t)(lt - s);
      ok = true;
    }
  } else if (tag == "<base64>") {
    const char* lt = (const char*)memchr(s + off, '<', len - off);  // binaryFromXml
    if (lt) {
      v.m_type = Value::BINARY;
      const size_t n = (size_t)(lt - (s + off));
      if (dst) {
        const long got = Base64Get(s + off, n, dst, cap);
        if (got >= 0) {
          *dst_len = (size_t)got;
          ok = true;
        }
      } else {
        v.m_bin.resize(n / 4 * 3 + 3);
        const long got = Base64Get(s + off, n, v.m_bin.empty() ? nullptr : &v.m_bin[0], v.m_bin.size());
        if (got >= 0) {
          v.m_bin.resize((size_t)got);
          ok = true;
        }
      }
      off = (size_t)(lt - s);
    }
  }
  if (ok) {
    const char* e = find(s, len, off, "</value>");  // findTag(VALUE_ETAG)
    if (e) off = (size_t)(e - s) + 8;
  } else {
    off = saved;
  }
  return ok;
}

}  // namespace

size_t Base64PutLength(size_t size) {
  const size_t full = size / 3;
  return 4 * full + (size % 3 ? 4 : 0) + full / 18;
}

void Base64Put(const U8* d, size_t n, std::string& out) {
  const size_t base = out.size();
  out.resize(base + Base64PutLength(n));
  char* o = &out[base];
  size_t i = 0;
  int line_groups = 0;
  for (; i + 3 <= n; i += 3) {
    const U32 x = ((U32)d[i] << 16) | ((U32)d[i + 1] << 8) | d[i + 2];
    *o++ = kAlphabet[x >> 18];
    *o++ = kAlphabet[(x >> 12) & 63];
    *o++ = kAlphabet[(x >> 6) & 63];
    *o++ = kAlphabet[x & 63];
    if (line_groups == 17) {  // base64.h:197-205: a newline after the 18th group
      *o++ = '\n';
      line_groups = 0;
    } else {
      ++line_groups;
    }
  }
  if (n - i == 1) {
    const U32 x = (U32)d[i] << 16;
    *o++ = kAlphabet[x >> 18];
    *o++ = kAlphabet[(x >> 12) & 63];
    *o++ = '=';
    *o++ = '=';
  } else if (n - i == 2) {
    const U32 x = ((U32)d[i] << 16) | ((U32)d[i + 1] << 8);
    *o++ = kAlphabet[x >> 18];
    *o++ = kAlphabet[(x >> 12) & 63];
    *o++ = kAlphabet[(x >> 6) & 63];
    *o++ = '=';
  }
}

long Base64Get(const char* t, size_t len, U8* out, size_t cap) {
  size_t p = 0, w = 0;
  // next character that is not skipped; kSkip at the end of input
  auto next = [&](U8& c) -> bool {
    while (p < len) {
      c = kDecode.v[(U8)t[p++]];
      if (c != kSkip) return true;
    }
    return false;
  };
  for (;;) {
    // fast path: four alphabet characters in a row
    if (p + 4 <= len) {
      const U8 a = kDecode.v[(U8)t[p]], b = kDecode.v[(U8)t[p + 1]], c = kDecode.v[(U8)t[p + 2]],
               e = kDecode.v[(U8)t[p + 3]];
      if ((a | b | c | e) < 64) {
        if (w + 3 > cap) return -1;
        const U32 x = ((U32)a << 18) | ((U32)b << 12) | ((U32)c << 6) | e;
        out[w] = (U8)(x >> 16);
        out[w + 1] = (U8)(x >> 8);
        out[w + 2] = (U8)x;
        w += 3;
        p += 4;
        continue;
      }
    }
    U8 c0, c1, c2, c3;
    if (!next(c0)) return (long)w;          // end between groups
    if (c0 == kEq) return (long)w;          // '=' cannot open a group
    if (!next(c1) || c1 == kEq) return (long)w;
    if (!next(c2)) return (long)w;          // group cut short: dropped
    if (c2 == kEq) {                        // "xx==": one byte, then stop
      if (w + 1 > cap) return -1;
      out[w++] = (U8)((c0 << 2) | (c1 >> 4));
      return (long)w;
    }
    if (!next(c3)) return (long)w;          // three characters then EOF: dropped
    if (c3 == kEq) {                        // "xxx=": two bytes, then stop
      if (w + 2 > cap) return -1;
      out[w++] = (U8)((c0 << 2) | (c1 >> 4));
      out[w++] = (U8)((c1 << 4) | (c2 >> 2));
      return (long)w;
    }
    if (w + 3 > cap) return -1;
    out[w++] = (U8)((c0 << 2) | (c1 >> 4));
    out[w++] = (U8)((c1 << 4) | (c2 >> 2));
    out[w++] = (U8)((c2 << 6) | c3);
  }
}

std::string XmlEncode(const std::string& raw) {
  std::string o;
  o.reserve(raw.size());
  for (char c : raw) {
    switch (c) {
      case '<': o += "&lt;"; break;
      case '>': o += "&gt;"; break;
      case '&': o += "&amp;"; break;
      case '\'': o += "&apos;"; break;
      case '"': o += "&quot;"; break;
      default: o += c;
    }
  }
  return o;
}

std::string XmlDecode(const std::string& enc) {
  static const char raw[] = {'<', '>', '&', '\'', '"'};
  static const char* ent[] = {"lt;", "gt;", "amp;", "apos;", "quot;"};
  std::string o;
  o.reserve(enc.size());
  for (size_t i = 0; i < enc.size();) {
    if (enc[i] == '&') {
      bool hit = false;
      for (int k = 0; k < 5; ++k) {
        const size_t n = strlen(ent[k]);
        if (enc.compare(i + 1, n, ent[k]) == 0) {
          o += raw[k];
          i += n + 1;
          hit = true;
          break;
        }
      }
      if (!hit) o += enc[i++];
    } else {
      o += enc[i++];
    }
  }
  return o;
}

std::string EncodeMethod(const std::string& method, const std::vector<Value>& params) {
  std::string body = kRequestBegin;
  body += method;
  body += kRequestEndMethodName;
  if (!params.empty()) {
    body += "<params>";
    for (const Value& v : params) {
      body += "<param>";
      value_xml(v, body);
      body += "</param>";
    }
    body += "</params>";
  }
  body += kRequestEnd;
  frame(body);
  return body;
}

std::string EncodeSendChunk(const std::string& filename, U32 index, const U8* data, U32 size) {
  char idx[32];
  snprintf(idx, sizeof(idx), "%d", (int)index);  // args[1] = (int)chunkindex, ChunkMethods.cpp:118-120
  std::string s;
  s.reserve(Base64PutLength(size) + filename.size() + 256);
  s += kRequestBegin;
  s += kSendChunk;
  s += kRequestEndMethodName;
  s += "<params><param><value>";
  s += XmlEncode(filename);
  s += "</value></param><param><value><i4>";
  s += idx;
  s += "</i4></value></param><param><value><base64>";
  Base64Put(data, size, s);
  s += "</base64></value></param></params>";
  s += kRequestEnd;
  frame(s);
  return s;
}

std::string FrameSendChunkText(const std::string& filename, U32 index, const char* text, size_t len) {
  char idx[32];
  snprintf(idx, sizeof(idx), "%d", (int)index);
  std::string s;
  s.reserve(len + filename.size() + 256);
  s += kRequestBegin;
  s += kSendChunk;
  s += kRequestEndMethodName;
  s += "<params><param><value>";
  s += XmlEncode(filename);
  s += "</value></param><param><value><i4>";
  s += idx;
  s += "</i4></value></param><param><value><base64>";
  for (char& c : s)  // frame()'s newline rule, for the header; the text has none
    if (c == '\n' || c == '\r') c = ' ';
  s.append(text, len);
  const size_t tail = s.size();
  s += "</base64></value></param></params>";
  s += kRequestEnd;
  for (size_t i = tail; i < s.size(); ++i)
    if (s[i] == '\n' || s[i] == '\r') s[i] = ' ';
  s += '\n';
  return s;
}

bool DecodeMethod(const std::string& f, std::string& o_method, std::vector<Value>& o_params) {
  o_params.clear();
  const char* s = f.data();
  const size_t len = f.size();
  // parseTag(METHODNAME_TAG)
  const char* a = find(s, len, 0, "<methodName>");
  if (!a) return false;
  const size_t b = (size_t)(a - s) + 12;
  const char* e = find(s, len, b, "</methodName>");
  if (!e) return false;
  o_method.assign(s + b, e);
  size_t off = (size_t)(e - s) + 13;
  if (o_method.empty()) return false;
  const char* pp = find(s, len, off, "<params>");  // findTag(PARAMS_TAG)
  if (!pp) return true;
  off = (size_t)(pp - s) + 8;
  while (next_tag_is("<param>", s, len, off)) {
    Value v;
    if (!parse_value(s, len, off, v, nullptr, 0, nullptr)) break;
    o_params.push_back(v);
    next_tag_is("</param>", s, len, off);
  }
  return true;
}

bool DecodeSendChunk(const char* s, size_t len, std::string& o_filename, U32& o_index, U8* dst, size_t cap,
                     size_t& o_size) {
  const char* a = find(s, len, 0, "<methodName>");
  if (!a) return false;
  const size_t b = (size_t)(a - s) + 12;
  const char* e = find(s, len, b, "</methodName>");
  if (!e || (size_t)(e - (s + b)) != strlen(kSendChunk) || memcmp(s + b, kSendChunk, strlen(kSendChunk)) != 0)
    return false;
  size_t off = (size_t)(e - s) + 13;
  const char* pp = find(s, len, off, "<params>");
  if (!pp) return false;
  off = (size_t)(pp - s) + 8;
  Value name, idx, data;
  if (!next_tag_is("<param>", s, len, off) || !parse_value(s, len, off, name, nullptr, 0, nullptr) ||
      name.m_type != Value::STRING)
    return false;
  next_tag_is("</param>", s, len, off);
  if (!next_tag_is("<param>", s, len, off) || !parse_value(s, len, off, idx, nullptr, 0, nullptr) ||
      idx.m_type != Value::INT)
    return false;
  next_tag_is("</param>", s, len, off);
  if (!next_tag_is("<param>", s, len, off) || !parse_value(s, len, off, data, dst, cap, &o_size) ||
      data.m_type != Value::BINARY)
    return false;
  o_filename = name.m_str;
  o_index = (U32)idx.m_int;
  return true;
}

bool LocateSendChunk(const char* s, size_t len, std::string& o_filename, U32& o_index, size_t& o_b64_offset,
                     size_t& o_b64_length) {
  const char* a = find(s, len, 0, "<methodName>");
  if (!a) return false;
  const size_t b = (size_t)(a - s) + 12;
  const char* e = find(s, len, b, "</methodName>");
  if (!e || (size_t)(e - (s + b)) != strlen(kSendChunk) || memcmp(s + b, kSendChunk, strlen(kSendChunk)) != 0)
    return false;
  size_t off = (size_t)(e - s) + 13;
  const char* pp = find(s, len, off, "<params>");
  if (!pp) return false;
  off = (size_t)(pp - s) + 8;
  Value name, idx;
  if (!next_tag_is("<param>", s, len, off) || !parse_value(s, len, off, name, nullptr, 0, nullptr) ||
      name.m_type != Value::STRING)
    return false;
  next_tag_is("</param>", s, len, off);
  if (!next_tag_is("<param>", s, len, off) || !parse_value(s, len, off, idx, nullptr, 0, nullptr) ||
      idx.m_type != Value::INT)
    return false;
  next_tag_is("</param>", s, len, off);
  // parse_value's <base64> branch (binaryFromXml), without the decode
  if (!next_tag_is("<param>", s, len, off) || !next_tag_is("<value>", s, len, off) ||
      get_next_tag(s, len, off) != "<base64>")
    return false;
  const char* lt = (const char*)memchr(s + off, '<', len - off);
  if (!lt) return false;
  o_b64_offset = off;
  o_b64_length = (size_t)(lt - (s + off));
  o_filename = name.m_str;
  o_index = (U32)idx.m_int;
  return true;
}

}  // namespace PeerWire
}  // namespace libBitFlood
