// json_min.cpp — recursive-descent JSON parser (RFC 8259 subset sufficient for
// the reference's serde_json scene files: objects, arrays, strings with escapes,
// numbers, true/false/null).
#include "json_min.h"

#include <stdio.h>

namespace fr {
namespace json {
namespace {

struct Parser {
  const char* p;
  const char* end;
  const char* begin;
  std::string err;
  int depth = 0;

  bool fail(const char* msg) {
    char buf[160];
    snprintf(buf, sizeof(buf), "json: %s at byte %ld", msg, static_cast<long>(p - begin));
    err = buf;
    return false;
  }
  void ws() {
    while (p < end && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  }
  bool lit(const char* s) {
    const char* q = p;
    while (*s) {
      if (q >= end || *q != *s) return false;
      ++q;
      ++s;
    }
    p = q;
    return true;
  }
  static void put_utf8(std::string& o, unsigned cp) {
    if (cp < 0x80) {
      o += static_cast<char>(cp);
    } else if (cp < 0x800) {
      o += static_cast<char>(0xC0 | (cp >> 6));
      o += static_cast<char>(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      o += static_cast<char>(0xE0 | (cp >> 12));
      o += static_cast<char>(0x80 | ((cp >> 6) & 0x3F));
      o += static_cast<char>(0x80 | (cp & 0x3F));
    } else {
      o += static_cast<char>(0xF0 | (cp >> 18));
      o += static_cast<char>(0x80 | ((cp >> 12) & 0x3F));
      o += static_cast<char>(0x80 | ((cp >> 6) & 0x3F));
      o += static_cast<char>(0x80 | (cp & 0x3F));
    }
  }
  bool hex4(unsigned& v) {
    v = 0;
    for (int i = 0; i < 4; ++i) {
      if (p >= end) return fail("truncated \\u escape");
      char c = *p++;
      v <<= 4;
      if (c >= '0' && c <= '9')
        v |= static_cast<unsigned>(c - '0');
      else if (c >= 'a' && c <= 'f')
        v |= static_cast<unsigned>(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F')
        v |= static_cast<unsigned>(c - 'A' + 10);
      else
        return fail("bad \\u escape");
    }
    return true;
  }
  bool str(std::string& o) {
    if (p >= end || *p != '"') return fail("expected string");
    ++p;
    while (true) {
      if (p >= end) return fail("unterminated string");
      char c = *p++;
      if (c == '"') return true;
      if (static_cast<unsigned char>(c) < 0x20) return fail("control character in string");
      if (c != '\\') {
        o += c;
        continue;
      }
      if (p >= end) return fail("truncated escape");
      char e = *p++;
      switch (e) {
        case '"': o += '"'; break;
        case '\\': o += '\\'; break;
        case '/': o += '/'; break;
        case 'b': o += '\b'; break;
        case 'f': o += '\f'; break;
        case 'n': o += '\n'; break;
        case 'r': o += '\r'; break;
        case 't': o += '\t'; break;
        case 'u': {
          unsigned cp;
          if (!hex4(cp)) return false;
          if (cp >= 0xD800 && cp < 0xDC00) {
            unsigned lo;
            if (!lit("\\u") || !hex4(lo) || lo < 0xDC00 || lo >= 0xE000) return fail("bad surrogate pair");
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          put_utf8(o, cp);
          break;
        }
        default: return fail("bad escape");
      }
    }
  }
  bool num(Value& v) {
    const char* s = p;
    if (p < end && *p == '-') ++p;
    if (p >= end) return fail("bad number");
    if (*p == '0') {
      ++p;
    } else if (*p >= '1' && *p <= '9') {
      while (p < end && *p >= '0' && *p <= '9') ++p;
    } else {
      return fail("bad number");
    }
    if (p < end && *p == '.') {
      ++p;
      if (p >= end || !(*p >= '0' && *p <= '9')) return fail("bad fraction");
      while (p < end && *p >= '0' && *p <= '9') ++p;
    }
    if (p < end && (*p == 'e' || *p == 'E')) {
      ++p;
      if (p < end && (*p == '+' || *p == '-')) ++p;
      if (p >= end || !(*p >= '0' && *p <= '9')) return fail("bad exponent");
      while (p < end && *p >= '0' && *p <= '9') ++p;
    }
    v.type = Value::Number;
    v.text.assign(s, p);
    return true;
  }
  bool value(Value& v) {
    if (++depth > 256) return fail("nesting too deep");
    ws();
    if (p >= end) return fail("unexpected end");
    bool ok;
    char c = *p;
    if (c == '{') {
      ok = object(v);
    } else if (c == '[') {
      ok = array(v);
    } else if (c == '"') {
      v.type = Value::String;
      ok = str(v.text);
    } else if (c == 't') {
      ok = lit("true") ? (v.type = Value::Bool, v.b = true, true) : fail("bad literal");
    } else if (c == 'f') {
      ok = lit("false") ? (v.type = Value::Bool, v.b = false, true) : fail("bad literal");
    } else if (c == 'n') {
      ok = lit("null") ? (v.type = Value::Null, true) : fail("bad literal");
    } else {
      ok = num(v);
    }
    --depth;
    return ok;
  }
  bool array(Value& v) {
    v.type = Value::Array;
    ++p;
    ws();
    if (p < end && *p == ']') {
      ++p;
      return true;
    }
    while (true) {
      v.items.emplace_back();
      if (!value(v.items.back())) return false;
      ws();
      if (p < end && *p == ',') {
        ++p;
        continue;
      }
      if (p < end && *p == ']') {
        ++p;
        return true;
      }
      return fail("expected , or ]");
    }
  }
  bool object(Value& v) {
    v.type = Value::Object;
    ++p;
    ws();
    if (p < end && *p == '}') {
      ++p;
      return true;
    }
    while (true) {
      ws();
      std::string key;
      if (!str(key)) return false;
      ws();
      if (p >= end || *p != ':') return fail("expected :");
      ++p;
      v.members.emplace_back(std::move(key), Value());
      if (!value(v.members.back().second)) return false;
      ws();
      if (p < end && *p == ',') {
        ++p;
        continue;
      }
      if (p < end && *p == '}') {
        ++p;
        return true;
      }
      return fail("expected , or }");
    }
  }
};

}  // namespace

bool parse(const char* text, size_t len, Value& out, std::string& err) {
  Parser ps{text, text + len, text};
  if (!ps.value(out)) {
    err = ps.err;
    return false;
  }
  ps.ws();
  if (ps.p != ps.end) {
    ps.fail("trailing characters");
    err = ps.err;
    return false;
  }
  return true;
}

}  // namespace json
}  // namespace fr
