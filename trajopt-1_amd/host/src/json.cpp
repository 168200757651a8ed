// Minimal JSON parser / DOM (see json.hpp).
#include "trajopt_amd/json.hpp"

#include <charconv>
#include <cmath>
#include <cstdlib>
#include <fstream>
#include <sstream>

namespace Json
{
namespace
{
const Value& nullRef()
{
  static const Value v;
  return v;
}

class Parser
{
public:
  explicit Parser(const std::string& s) : s_(s) {}

  Value document()
  {
    skipWs();
    Value v = value(0);
    skipWs();
    if (pos_ != s_.size())
      fail("trailing characters after the document");
    return v;
  }

private:
  [[noreturn]] void fail(const std::string& what) const
  {
    int line = 1, col = 1;
    for (std::size_t i = 0; i < pos_ && i < s_.size(); ++i)
    {
      if (s_[i] == '\n')
      {
        ++line;
        col = 1;
      }
      else
        ++col;
    }
    throw std::runtime_error("json: " + what + " at line " + std::to_string(line) + " col " + std::to_string(col));
  }

  void skipWs()
  {
    while (pos_ < s_.size())
    {
      const char c = s_[pos_];
      if (c == ' ' || c == '\t' || c == '\n' || c == '\r')
        ++pos_;
      else if (c == '/' && pos_ + 1 < s_.size() && s_[pos_ + 1] == '/')  // jsoncpp accepts comments
      {
        while (pos_ < s_.size() && s_[pos_] != '\n')
          ++pos_;
      }
      else
        break;
    }
  }

  bool consume(char c)
  {
    if (pos_ < s_.size() && s_[pos_] == c)
    {
      ++pos_;
      return true;
    }
    return false;
  }

  void expectWord(const char* w)
  {
    for (const char* p = w; *p; ++p)
      if (!consume(*p))
        fail(std::string("invalid literal, expected '") + w + "'");
  }

  Value value(int depth)
  {
    if (depth > 256)
      fail("nesting too deep");
    if (pos_ >= s_.size())
      fail("unexpected end of input");
    const char c = s_[pos_];
    if (c == '{')
      return object(depth);
    if (c == '[')
      return array(depth);
    if (c == '"')
      return Value(string());
    if (c == 't')
    {
      expectWord("true");
      return Value(true);
    }
    if (c == 'f')
    {
      expectWord("false");
      return Value(false);
    }
    if (c == 'n')
    {
      expectWord("null");
      return Value();
    }
    if (c == '-' || (c >= '0' && c <= '9'))
      return number();
    fail(std::string("unexpected character '") + c + "'");
  }

  // Number tokens as the reference's parser reads them (Json::Reader,
  // trajopt/test/trajopt_test_utils.hpp:14; jsoncpp Reader::readNumber /
  // decodeNumber / decodeDouble): an optional '-', digits, an optional '.' and
  // digits, an optional exponent, each part possibly empty.  A token of only
  // '-' and digits is an integer ("01" -> 1, "-" -> 0); any other token must
  // convert as a whole to a finite double ("1." -> 1, "-.5" -> -0.5; "1e",
  // "1e999" fail).  The conversion is std::from_chars, which ignores the C
  // locale (strtod would read "0.5" as 0 under a comma-decimal LC_NUMERIC).
  Value number()
  {
    const std::size_t start = pos_;
    auto digit = [&](std::size_t p) { return p < s_.size() && s_[p] >= '0' && s_[p] <= '9'; };
    std::size_t p = pos_;
    if (p < s_.size() && s_[p] == '-')
      ++p;
    const std::size_t int0 = p;
    while (digit(p))
      ++p;
    bool integral = true;
    if (p < s_.size() && s_[p] == '.')
    {
      integral = false;
      ++p;
      while (digit(p))
        ++p;
    }
    if (p < s_.size() && (s_[p] == 'e' || s_[p] == 'E'))
    {
      integral = false;
      ++p;
      if (p < s_.size() && (s_[p] == '+' || s_[p] == '-'))
        ++p;
      while (digit(p))
        ++p;
    }
    const char* first = s_.data() + start;
    const char* last = s_.data() + p;
    double d = 0.0;
    if (integral)
    {
      unsigned long long u = 0;
      const auto r = std::from_chars(s_.data() + int0, last, u);
      if (int0 == p)
        u = 0;  // "-": jsoncpp decodes an empty digit run as 0
      else if (r.ec == std::errc::result_out_of_range)
        integral = false;  // beyond 64 bits: jsoncpp falls back to decodeDouble
      if (integral)
      {
        d = static_cast<double>(u);
        if (s_[start] == '-')
          d = -d;
      }
    }
    if (!integral)
    {
      const auto r = std::from_chars(first, last, d);
      if (r.ec == std::errc::result_out_of_range || !std::isfinite(d))
        fail("number out of range");
      if (r.ec != std::errc() || r.ptr != last)
        fail("invalid number");
    }
    pos_ = p;
    return Value(d);
  }

  static void putUtf8(std::string& out, unsigned cp)
  {
    if (cp < 0x80)
      out += static_cast<char>(cp);
    else if (cp < 0x800)
    {
      out += static_cast<char>(0xC0 | (cp >> 6));
      out += static_cast<char>(0x80 | (cp & 0x3F));
    }
    else
    {
      out += static_cast<char>(0xE0 | (cp >> 12));
      out += static_cast<char>(0x80 | ((cp >> 6) & 0x3F));
      out += static_cast<char>(0x80 | (cp & 0x3F));
    }
  }

  std::string string()
  {
    consume('"');
    std::string out;
    while (true)
    {
      if (pos_ >= s_.size())
        fail("unterminated string");
      const char c = s_[pos_++];
      if (c == '"')
        break;
      if (c != '\\')
      {
        out += c;
        continue;
      }
      if (pos_ >= s_.size())
        fail("unterminated escape");
      const char e = s_[pos_++];
      switch (e)
      {
        case '"':
        case '\\':
        case '/':
          out += e;
          break;
        case 'b':
          out += '\b';
          break;
        case 'f':
          out += '\f';
          break;
        case 'n':
          out += '\n';
          break;
        case 'r':
          out += '\r';
          break;
        case 't':
          out += '\t';
          break;
        case 'u':
        {
          if (pos_ + 4 > s_.size())
            fail("bad \\u escape");
          unsigned cp = 0;
          for (int i = 0; i < 4; ++i)
          {
            const char h = s_[pos_++];
            cp <<= 4;
            if (h >= '0' && h <= '9')
              cp |= static_cast<unsigned>(h - '0');
            else if (h >= 'a' && h <= 'f')
              cp |= static_cast<unsigned>(h - 'a' + 10);
            else if (h >= 'A' && h <= 'F')
              cp |= static_cast<unsigned>(h - 'A' + 10);
            else
              fail("bad \\u escape");
          }
          putUtf8(out, cp);
          break;
        }
        default:
          fail("bad escape");
      }
    }
    return out;
  }

  Value array(int depth)
  {
    consume('[');
    Value v(Value::arrayValue);
    skipWs();
    if (consume(']'))
      return v;
    while (true)
    {
      skipWs();
      v.append(value(depth + 1));
      skipWs();
      if (consume(']'))
        return v;
      if (!consume(','))
        fail("expected ',' or ']'");
    }
  }

  Value object(int depth)
  {
    consume('{');
    Value v(Value::objectValue);
    skipWs();
    if (consume('}'))
      return v;
    while (true)
    {
      skipWs();
      if (pos_ >= s_.size() || s_[pos_] != '"')
        fail("expected a member name");
      std::string key = string();
      skipWs();
      if (!consume(':'))
        fail("expected ':'");
      skipWs();
      v.set(key, value(depth + 1));
      skipWs();
      if (consume('}'))
        return v;
      if (!consume(','))
        fail("expected ',' or '}'");
    }
  }

  const std::string& s_;
  std::size_t pos_ = 0;
};

void styled(const Value& v, std::ostringstream& os)
{
  switch (v.type())
  {
    case Value::nullValue:
      os << "null";
      break;
    case Value::boolValue:
      os << (v.asBool() ? "true" : "false");
      break;
    case Value::numberValue:
    {
      std::ostringstream t;
      t.precision(17);
      t << v.asDouble();
      os << t.str();
      break;
    }
    case Value::stringValue:
      os << '"' << v.asString() << '"';
      break;
    case Value::arrayValue:
    {
      os << '[';
      bool first = true;
      for (const auto& e : v)
      {
        if (!first)
          os << ", ";
        first = false;
        styled(e, os);
      }
      os << ']';
      break;
    }
    case Value::objectValue:
    {
      os << '{';
      const auto names = v.getMemberNames();
      for (std::size_t i = 0; i < names.size(); ++i)
      {
        if (i)
          os << ", ";
        os << '"' << names[i] << "\": ";
        styled(v[names[i]], os);
      }
      os << '}';
      break;
    }
  }
}
}  // namespace

bool Value::asBool() const
{
  if (type_ == boolValue)
    return b_;
  if (type_ == numberValue)
    return num_ != 0.0;
  if (type_ == nullValue)
    return false;
  throw std::runtime_error("json: value is not convertible to bool");
}

double Value::asDouble() const
{
  if (type_ == numberValue)
    return num_;
  if (type_ == boolValue)
    return b_ ? 1.0 : 0.0;
  if (type_ == nullValue)
    return 0.0;
  throw std::runtime_error("json: value is not convertible to double");
}

int Value::asInt() const
{
  const double d = asDouble();
  if (d != std::floor(d) || d < -2147483648.0 || d > 2147483647.0)
    throw std::runtime_error("json: value is not an int: " + toStyledString());
  return static_cast<int>(d);
}

const std::string& Value::asString() const
{
  if (type_ != stringValue)
    throw std::runtime_error("json: value is not a string: " + toStyledString());
  return str_;
}

std::size_t Value::size() const { return (type_ == arrayValue || type_ == objectValue) ? items_.size() : 0; }

bool Value::isMember(const std::string& key) const
{
  if (type_ != objectValue)
    return false;
  for (const auto& k : keys_)
    if (k == key)
      return true;
  return false;
}

const Value& Value::operator[](const std::string& key) const
{
  if (type_ == objectValue)
    for (std::size_t i = 0; i < keys_.size(); ++i)
      if (keys_[i] == key)
        return items_[i];
  return nullRef();
}

const Value& Value::operator[](std::size_t i) const
{
  if (type_ == arrayValue && i < items_.size())
    return items_[i];
  return nullRef();
}

std::vector<std::string> Value::getMemberNames() const { return type_ == objectValue ? keys_ : std::vector<std::string>{}; }

Value& Value::append(Value v)
{
  if (type_ == nullValue)
    type_ = arrayValue;
  if (type_ != arrayValue)
    throw std::runtime_error("json: append on a non-array");
  items_.push_back(std::move(v));
  return items_.back();
}

Value& Value::set(const std::string& key, Value v)
{
  if (type_ == nullValue)
    type_ = objectValue;
  if (type_ != objectValue)
    throw std::runtime_error("json: set on a non-object");
  for (std::size_t i = 0; i < keys_.size(); ++i)
    if (keys_[i] == key)  // duplicate member: last one wins (jsoncpp)
      return items_[i] = std::move(v);
  keys_.push_back(key);
  items_.push_back(std::move(v));
  return items_.back();
}

std::string Value::toStyledString() const
{
  std::ostringstream os;
  styled(*this, os);
  return os.str();
}

Value parse(const std::string& text) { return Parser(text).document(); }

Value parseFile(const std::string& path)
{
  std::ifstream f(path);
  if (!f)
    throw std::runtime_error("json: cannot open " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  return parse(ss.str());
}
}  // namespace Json

namespace json_marshal
{
void fromJson(const Json::Value& v, bool& ref)
{
  if (!v.isBool() && !v.isNumeric())
    throw std::runtime_error("expected bool, got " + v.toStyledString());
  ref = v.asBool();
}
void fromJson(const Json::Value& v, int& ref)
{
  if (!v.isNumeric())
    throw std::runtime_error("expected int, got " + v.toStyledString());
  ref = v.asInt();
}
void fromJson(const Json::Value& v, double& ref)
{
  if (!v.isNumeric())
    throw std::runtime_error("expected double, got " + v.toStyledString());
  ref = v.asDouble();
}
void fromJson(const Json::Value& v, std::string& ref)
{
  if (!v.isString())
    throw std::runtime_error("expected string, got " + v.toStyledString());
  ref = v.asString();
}
}  // namespace json_marshal
