#include "proto.hpp"

#include <cctype>
#include <cstdlib>
#include <fstream>
#include <sstream>

namespace caffe {

namespace {

class Lexer {
 public:
  explicit Lexer(const std::string& s) : s_(s) {}

  [[noreturn]] void fail(const std::string& what) const {
    std::ostringstream o;
    o << "prototxt parse error at line " << line_ << ", column " << col_ << ": " << what;
    throw std::runtime_error(o.str());
  }

  void skip() {
    while (i_ < s_.size()) {
      char c = s_[i_];
      if (c == '#') {
        while (i_ < s_.size() && s_[i_] != '\n') adv();
      } else if (std::isspace(static_cast<unsigned char>(c)) || c == ',' || c == ';') {
        adv();
      } else {
        break;
      }
    }
  }
  bool eof() {
    skip();
    return i_ >= s_.size();
  }
  char peek() {
    skip();
    return i_ < s_.size() ? s_[i_] : '\0';
  }
  void expect(char c) {
    if (peek() != c) fail(std::string("expected '") + c + "'");
    adv();
  }
  bool accept(char c) {
    if (peek() == c) {
      adv();
      return true;
    }
    return false;
  }
  std::string ident() {
    skip();
    size_t st = i_;
    while (i_ < s_.size() && (std::isalnum(static_cast<unsigned char>(s_[i_])) || s_[i_] == '_' ||
                              s_[i_] == '.' || s_[i_] == '-' || s_[i_] == '+'))
      adv();
    if (st == i_) fail("expected identifier or number");
    return s_.substr(st, i_ - st);
  }
  std::string quoted() {
    skip();
    char q = s_[i_];
    adv();
    std::string out;
    while (i_ < s_.size() && s_[i_] != q) {
      char c = s_[i_];
      if (c == '\\' && i_ + 1 < s_.size()) {
        adv();
        char e = s_[i_];
        switch (e) {
          case 'n': out += '\n'; break;
          case 't': out += '\t'; break;
          default: out += e;
        }
      } else {
        out += c;
      }
      adv();
    }
    if (i_ >= s_.size()) fail("unterminated string");
    adv();
    return out;
  }

 private:
  void adv() {
    if (s_[i_] == '\n') {
      ++line_;
      col_ = 1;
    } else {
      ++col_;
    }
    ++i_;
  }
  const std::string& s_;
  size_t i_ = 0;
  int line_ = 1, col_ = 1;
};

// protobuf's text parser stops at 100 levels of nesting (its default
// recursion limit); deeper input is rejected instead of exhausting the stack
constexpr int kMaxDepth = 100;

void parse_body(Lexer& lx, Msg& m, bool top, int depth = 0) {
  if (depth > kMaxDepth) lx.fail("message nesting deeper than 100 levels");
  while (true) {
    if (top) {
      if (lx.eof()) return;
    } else if (lx.peek() == '}') {
      return;
    } else if (lx.eof()) {
      lx.fail("unexpected end of input inside message");
    }
    std::string key = lx.ident();
    Value v;
    bool colon = lx.accept(':');
    char c = lx.peek();
    if (c == '{' || c == '<') {
      char close = (c == '{') ? '}' : '>';
      lx.expect(c);
      v.is_msg = true;
      v.msg = std::make_shared<Msg>();
      parse_body(lx, *v.msg, false, depth + 1);
      lx.expect(close);
    } else {
      if (!colon) lx.fail("expected ':' after field '" + key + "'");
      if (c == '"' || c == '\'') {
        v.quoted = true;
        v.scalar = lx.quoted();
        // adjacent string literals concatenate
        while (lx.peek() == '"' || lx.peek() == '\'') v.scalar += lx.quoted();
      } else if (c == '[') {
        // repeated scalar list: key: [a, b, c]
        lx.expect('[');
        while (!lx.accept(']')) {
          Value e;
          if (lx.peek() == '"' || lx.peek() == '\'') {
            e.quoted = true;
            e.scalar = lx.quoted();
          } else {
            e.scalar = lx.ident();
          }
          m.fields.emplace_back(key, e);
        }
        continue;
      } else {
        v.scalar = lx.ident();
      }
    }
    m.fields.emplace_back(key, v);
  }
}

}  // namespace

bool Msg::has(const std::string& k) const { return first(k) != nullptr; }
int Msg::count(const std::string& k) const {
  int n = 0;
  for (auto& f : fields) n += (f.first == k);
  return n;
}
const Value* Msg::first(const std::string& k) const {
  for (auto& f : fields)
    if (f.first == k) return &f.second;
  return nullptr;
}
std::vector<const Value*> Msg::all(const std::string& k) const {
  std::vector<const Value*> r;
  for (auto& f : fields)
    if (f.first == k) r.push_back(&f.second);
  return r;
}
std::string Msg::str(const std::string& k, const std::string& def) const {
  // a non-repeated field set twice: protobuf keeps the last value
  const Value* v = nullptr;
  for (auto& f : fields)
    if (f.first == k) v = &f.second;
  if (!v || v->is_msg) return def;
  return v->scalar;
}
static double to_num(const std::string& s, const std::string& k) {
  if (s == "true") return 1.0;
  if (s == "false") return 0.0;
  if (s == "inf" || s == "infinity") return 1e300 * 1e300;
  if (s == "-inf") return -(1e300 * 1e300);
  char* end = nullptr;
  std::string t = s;
  if (!t.empty() && (t.back() == 'f' || t.back() == 'F') && t.find_first_of("xX") == std::string::npos)
    t.pop_back();
  double d = std::strtod(t.c_str(), &end);
  if (end == t.c_str() || *end != '\0') throw std::runtime_error("field '" + k + "': not a number: " + s);
  return d;
}
double Msg::num(const std::string& k, double def) const {
  const Value* v = nullptr;
  for (auto& f : fields)
    if (f.first == k) v = &f.second;
  if (!v || v->is_msg) return def;
  return to_num(v->scalar, k);
}
long long Msg::integer(const std::string& k, long long def) const {
  const double d = num(k, static_cast<double>(def));
  // out-of-range (or NaN) -> error, never an undefined float->int conversion
  if (!(d >= -9.2e18 && d <= 9.2e18)) throw std::runtime_error("field '" + k + "': integer out of range");
  return static_cast<long long>(d);
}
bool Msg::boolean(const std::string& k, bool def) const {
  std::string s = str(k, def ? "true" : "false");
  return s == "true" || s == "1" || s == "True";
}
std::vector<double> Msg::nums(const std::string& k) const {
  std::vector<double> r;
  for (auto* v : all(k))
    if (!v->is_msg) r.push_back(to_num(v->scalar, k));
  return r;
}
std::vector<std::string> Msg::strs(const std::string& k) const {
  std::vector<std::string> r;
  for (auto* v : all(k))
    if (!v->is_msg) r.push_back(v->scalar);
  return r;
}
const Msg* Msg::sub(const std::string& k) const {
  const Value* v = nullptr;
  for (auto& f : fields)
    if (f.first == k && f.second.is_msg) v = &f.second;
  return v ? v->msg.get() : nullptr;
}
std::vector<const Msg*> Msg::subs(const std::string& k) const {
  std::vector<const Msg*> r;
  for (auto* v : all(k))
    if (v->is_msg) r.push_back(v->msg.get());
  return r;
}
const Msg& Msg::sub_or_empty(const std::string& k) const {
  static const Msg empty;
  const Msg* m = sub(k);
  return m ? *m : empty;
}
void Msg::set(const std::string& k, const std::string& v, bool quoted) {
  for (auto& f : fields)
    if (f.first == k && !f.second.is_msg) {
      f.second.scalar = v;
      f.second.quoted = quoted;
      return;
    }
  Value val;
  val.scalar = v;
  val.quoted = quoted;
  fields.emplace_back(k, val);
}
void Msg::add(const std::string& k, const std::string& v, bool quoted) {
  Value val;
  val.scalar = v;
  val.quoted = quoted;
  fields.emplace_back(k, val);
}
Msg& Msg::add_sub(const std::string& k) {
  Value v;
  v.is_msg = true;
  v.msg = std::make_shared<Msg>();
  fields.emplace_back(k, v);
  return *fields.back().second.msg;
}
std::string Msg::debug_string(int indent) const {
  std::ostringstream o;
  std::string pad(indent, ' ');
  for (auto& f : fields) {
    if (f.second.is_msg) {
      o << pad << f.first << " {\n" << f.second.msg->debug_string(indent + 2) << pad << "}\n";
    } else if (f.second.quoted) {
      o << pad << f.first << ": \"" << f.second.scalar << "\"\n";
    } else {
      o << pad << f.first << ": " << f.second.scalar << "\n";
    }
  }
  return o.str();
}

Msg parse_prototxt(const std::string& text) {
  Lexer lx(text);
  Msg m;
  parse_body(lx, m, true);
  return m;
}

Msg parse_prototxt_file(const std::string& path) {
  std::ifstream f(path);
  if (!f) throw std::runtime_error("cannot open prototxt file: " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  return parse_prototxt(ss.str());
}

}  // namespace caffe
