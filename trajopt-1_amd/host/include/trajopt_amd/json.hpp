// Minimal JSON document model for the problem front door.
//
// The reference reads problems with jsoncpp (Json::Value) through the helpers
// of trajopt/include/trajopt/json_marshal.hpp:17-86; jsoncpp is not in this
// image, so this is a small DOM with the subset of the Json::Value interface
// the front door uses (isMember, operator[], size, iteration, as*()), plus
// json_marshal's childFromJson / fromJsonArray semantics (missing required
// field -> "missing field: <name>", default otherwise).
#pragma once
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace Json
{
class Value
{
public:
  enum Type
  {
    nullValue,
    boolValue,
    numberValue,
    stringValue,
    arrayValue,
    objectValue
  };

  Value() = default;
  explicit Value(Type t) : type_(t) {}
  explicit Value(double d) : type_(numberValue), num_(d) {}
  explicit Value(bool b) : type_(boolValue), b_(b) {}
  explicit Value(std::string s) : type_(stringValue), str_(std::move(s)) {}

  Type type() const { return type_; }
  bool isNull() const { return type_ == nullValue; }
  bool isBool() const { return type_ == boolValue; }
  bool isNumeric() const { return type_ == numberValue; }
  bool isString() const { return type_ == stringValue; }
  bool isArray() const { return type_ == arrayValue; }
  bool isObject() const { return type_ == objectValue; }

  bool asBool() const;
  double asDouble() const;
  int asInt() const;
  const std::string& asString() const;

  // arrays: element count; objects: member count; otherwise 0
  std::size_t size() const;
  bool isMember(const std::string& key) const;
  // missing members / out-of-range indices read as a shared null value
  const Value& operator[](const std::string& key) const;
  const Value& operator[](std::size_t i) const;
  const Value& operator[](int i) const { return (*this)[static_cast<std::size_t>(i)]; }
  std::vector<std::string> getMemberNames() const;  // document order

  // iteration over array elements or object member values (document order)
  const std::vector<Value>& elements() const { return items_; }
  std::vector<Value>::const_iterator begin() const { return items_.begin(); }
  std::vector<Value>::const_iterator end() const { return items_.end(); }

  // building
  Value& append(Value v);
  Value& set(const std::string& key, Value v);

  std::string toStyledString() const;

private:
  Type type_{ nullValue };
  double num_{ 0 };
  bool b_{ false };
  std::string str_;
  std::vector<Value> items_;        // array elements / object values
  std::vector<std::string> keys_;   // object keys (parallel to items_)
};

// Parses a complete JSON text; throws std::runtime_error("json: ... at line L col C").
Value parse(const std::string& text);
Value parseFile(const std::string& path);
}  // namespace Json

namespace json_marshal
{
// json_marshal.hpp:17-86 restated on Json::Value
void fromJson(const Json::Value& v, bool& ref);
void fromJson(const Json::Value& v, int& ref);
void fromJson(const Json::Value& v, double& ref);
void fromJson(const Json::Value& v, std::string& ref);

template <class T>
void fromJsonArray(const Json::Value& parent, std::vector<T>& ref)
{
  ref.clear();
  ref.reserve(parent.size());
  for (const auto& it : parent)
  {
    T t;
    fromJson(it, t);
    ref.push_back(t);
  }
}

template <class T>
void fromJsonArray(const Json::Value& parent, std::vector<T>& ref, int size)
{
  if (static_cast<int>(parent.size()) != size)
    throw std::runtime_error("expected list of size size " + std::to_string(size) +
                             ". got: " + parent.toStyledString());
  fromJsonArray(parent, ref);
}

template <class T>
void fromJson(const Json::Value& v, std::vector<T>& ref)
{
  fromJsonArray(v, ref);
}

template <class T>
void childFromJson(const Json::Value& parent, T& ref, const char* name, const T& df)
{
  if (parent.isMember(name))
    fromJson(parent[name], ref);
  else
    ref = df;
}

template <class T>
void childFromJson(const Json::Value& parent, T& ref, const char* name)
{
  if (parent.isMember(name))
    fromJson(parent[name], ref);
  else
    throw std::runtime_error(std::string("missing field: ") + name);
}
}  // namespace json_marshal
