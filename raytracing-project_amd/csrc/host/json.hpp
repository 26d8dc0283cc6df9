// json.hpp — a small strict JSON DOM for the scene loader.
//
// The reference parses scenes with nlohmann::json (raytracer/src/json_loader.cpp:21-22),
// which is not available here.  This parser reproduces the parts of nlohmann's
// behaviour that the loader can observe:
//   * RFC 8259 strict syntax: no comments, no trailing commas, no NaN/Infinity,
//     a leading UTF-8 BOM is skipped, trailing non-whitespace is an error;
//   * numbers: an integer literal is number_unsigned (>= 0) or number_integer
//     (< 0) when it fits 64 bits, otherwise number_float; "-0" is integer 0;
//   * objects behave like std::map: unique keys, the last duplicate wins;
//   * contains(key) on a non-object is false; at(key) on a non-object throws;
//   * get<int>  accepts number_* and boolean (static_cast);
//     get<double> accepts number_* only; get<string> accepts strings only.
// Error messages use nlohmann's "[json.exception.*]" wording.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace rtjson {

struct parse_error : std::runtime_error {
    using std::runtime_error::runtime_error;
};
struct type_error : std::runtime_error {
    using std::runtime_error::runtime_error;
};
struct out_of_range : std::runtime_error {
    using std::runtime_error::runtime_error;
};

class Value {
public:
    enum class Type { Null, Object, Array, String, Boolean, Integer, Unsigned, Float };

    Value() = default;

    Type type() const { return type_; }
    const char* type_name() const;

    bool is_object() const { return type_ == Type::Object; }
    bool is_array() const { return type_ == Type::Array; }
    bool is_string() const { return type_ == Type::String; }
    bool is_number() const {
        return type_ == Type::Integer || type_ == Type::Unsigned || type_ == Type::Float;
    }

    // Container size like nlohmann::json::size(): null 0, scalars 1.
    size_t size() const;
    bool empty() const { return size() == 0; }

    bool contains(const std::string& key) const;
    const Value& at(const std::string& key) const;
    const Value& at(size_t idx) const;
    const Value& operator[](size_t idx) const { return at(idx); }

    // Typed getters with nlohmann's conversion rules.
    double get_double() const;
    int get_int() const;
    std::string get_string() const;

    const std::vector<Value>& array_items() const { return arr_; }
    const std::map<std::string, Value>& object_items() const { return obj_; }

    static Value parse(const std::string& text);

private:
    friend class Parser;
    Type type_ = Type::Null;
    bool b_ = false;
    int64_t i_ = 0;
    uint64_t u_ = 0;
    double d_ = 0.0;
    std::string s_;
    std::vector<Value> arr_;
    std::map<std::string, Value> obj_;
};

}  // namespace rtjson
