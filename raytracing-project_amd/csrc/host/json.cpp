// json.cpp — strict recursive-descent JSON parser (see json.hpp for the
// nlohmann-compatible semantics it reproduces).
#include "json.hpp"

#include <cerrno>
#include <clocale>
#include <cstdlib>
#include <cstring>
#include <sstream>

namespace rtjson {

const char* Value::type_name() const {
    switch (type_) {
        case Type::Null: return "null";
        case Type::Object: return "object";
        case Type::Array: return "array";
        case Type::String: return "string";
        case Type::Boolean: return "boolean";
        default: return "number";
    }
}

size_t Value::size() const {
    switch (type_) {
        case Type::Null: return 0;
        case Type::Object: return obj_.size();
        case Type::Array: return arr_.size();
        default: return 1;
    }
}

bool Value::contains(const std::string& key) const {
    return type_ == Type::Object && obj_.count(key) != 0;
}

const Value& Value::at(const std::string& key) const {
    if (type_ != Type::Object)
        throw type_error(std::string("[json.exception.type_error.304] cannot use at() with ") +
                         type_name());
    auto it = obj_.find(key);
    if (it == obj_.end())
        throw out_of_range("[json.exception.out_of_range.403] key '" + key + "' not found");
    return it->second;
}

const Value& Value::at(size_t idx) const {
    if (type_ != Type::Array)
        throw type_error(std::string("[json.exception.type_error.304] cannot use at() with ") +
                         type_name());
    if (idx >= arr_.size())
        throw out_of_range("[json.exception.out_of_range.401] array index " + std::to_string(idx) +
                           " is out of range");
    return arr_[idx];
}

double Value::get_double() const {
    switch (type_) {
        case Type::Unsigned: return static_cast<double>(u_);
        case Type::Integer: return static_cast<double>(i_);
        case Type::Float: return d_;
        default:
            throw type_error(std::string("[json.exception.type_error.302] type must be number, but is ") +
                             type_name());
    }
}

int Value::get_int() const {
    switch (type_) {
        case Type::Unsigned: return static_cast<int>(u_);
        case Type::Integer: return static_cast<int>(i_);
        case Type::Float: return static_cast<int>(d_);
        case Type::Boolean: return static_cast<int>(b_);
        default:
            throw type_error(std::string("[json.exception.type_error.302] type must be number, but is ") +
                             type_name());
    }
}

std::string Value::get_string() const {
    if (type_ != Type::String)
        throw type_error(std::string("[json.exception.type_error.302] type must be string, but is ") +
                         type_name());
    return s_;
}

// ------------------------------------------------------------------ parser
class Parser {
public:
    explicit Parser(const std::string& t) : s_(t), n_(t.size()) {}

    Value parse_document() {
        // nlohmann skips a UTF-8 byte-order mark at the start of the input.
        if (n_ >= 3 && (unsigned char)s_[0] == 0xEF && (unsigned char)s_[1] == 0xBB &&
            (unsigned char)s_[2] == 0xBF)
            pos_ = 3;
        skip_ws();
        if (pos_ >= n_) fail("syntax error while parsing value - unexpected end of input");
        Value v = parse_value(0);
        skip_ws();
        if (pos_ != n_) fail("syntax error while parsing value - unexpected trailing content; expected end of input");
        return v;
    }

private:
    const std::string& s_;
    size_t n_;
    size_t pos_ = 0;

    [[noreturn]] void fail(const std::string& what) const {
        size_t line = 1, col = 0;
        for (size_t i = 0; i < pos_ && i < n_; ++i) {
            if (s_[i] == '\n') { ++line; col = 0; } else { ++col; }
        }
        std::ostringstream os;
        os << "[json.exception.parse_error.101] parse error at line " << line << ", column "
           << (col + 1) << ": " << what;
        throw parse_error(os.str());
    }

    void skip_ws() {
        while (pos_ < n_) {
            char c = s_[pos_];
            if (c == ' ' || c == '\t' || c == '\n' || c == '\r') ++pos_;
            else break;
        }
    }

    Value parse_value(int depth) {
        if (depth > 4096) fail("nesting too deep");
        skip_ws();
        if (pos_ >= n_) fail("syntax error while parsing value - unexpected end of input");
        char c = s_[pos_];
        switch (c) {
            case '{': return parse_object(depth);
            case '[': return parse_array(depth);
            case '"': {
                Value v;
                v.type_ = Value::Type::String;
                v.s_ = parse_string();
                return v;
            }
            case 't': expect_literal("true"); { Value v; v.type_ = Value::Type::Boolean; v.b_ = true; return v; }
            case 'f': expect_literal("false"); { Value v; v.type_ = Value::Type::Boolean; v.b_ = false; return v; }
            case 'n': expect_literal("null"); return Value();
            default:
                if (c == '-' || (c >= '0' && c <= '9')) return parse_number();
                fail("syntax error while parsing value - invalid literal");
        }
    }

    void expect_literal(const char* lit) {
        size_t L = std::strlen(lit);
        if (pos_ + L > n_ || s_.compare(pos_, L, lit) != 0)
            fail("syntax error while parsing value - invalid literal");
        pos_ += L;
    }

    Value parse_object(int depth) {
        Value v;
        v.type_ = Value::Type::Object;
        ++pos_;  // '{'
        skip_ws();
        if (pos_ < n_ && s_[pos_] == '}') { ++pos_; return v; }
        for (;;) {
            skip_ws();
            if (pos_ >= n_ || s_[pos_] != '"')
                fail("syntax error while parsing object key - invalid literal; expected string literal");
            std::string key = parse_string();
            skip_ws();
            if (pos_ >= n_ || s_[pos_] != ':')
                fail("syntax error while parsing object separator - expected ':'");
            ++pos_;
            Value child = parse_value(depth + 1);
            v.obj_[key] = std::move(child);  // std::map: the last duplicate wins
            skip_ws();
            if (pos_ >= n_) fail("syntax error while parsing object - unexpected end of input; expected '}'");
            if (s_[pos_] == ',') { ++pos_; continue; }
            if (s_[pos_] == '}') { ++pos_; return v; }
            fail("syntax error while parsing object - unexpected character; expected '}'");
        }
    }

    Value parse_array(int depth) {
        Value v;
        v.type_ = Value::Type::Array;
        ++pos_;  // '['
        skip_ws();
        if (pos_ < n_ && s_[pos_] == ']') { ++pos_; return v; }
        for (;;) {
            v.arr_.push_back(parse_value(depth + 1));
            skip_ws();
            if (pos_ >= n_) fail("syntax error while parsing array - unexpected end of input; expected ']'");
            if (s_[pos_] == ',') { ++pos_; continue; }
            if (s_[pos_] == ']') { ++pos_; return v; }
            fail("syntax error while parsing array - unexpected character; expected ']'");
        }
    }

    static void append_utf8(std::string& out, uint32_t cp) {
        if (cp < 0x80) {
            out.push_back((char)cp);
        } else if (cp < 0x800) {
            out.push_back((char)(0xC0 | (cp >> 6)));
            out.push_back((char)(0x80 | (cp & 0x3F)));
        } else if (cp < 0x10000) {
            out.push_back((char)(0xE0 | (cp >> 12)));
            out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
            out.push_back((char)(0x80 | (cp & 0x3F)));
        } else {
            out.push_back((char)(0xF0 | (cp >> 18)));
            out.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
            out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
            out.push_back((char)(0x80 | (cp & 0x3F)));
        }
    }

    uint32_t parse_hex4() {
        if (pos_ + 4 > n_) fail("syntax error while parsing value - invalid string: '\\u' must be followed by 4 hex digits");
        uint32_t v = 0;
        for (int k = 0; k < 4; ++k) {
            char c = s_[pos_++];
            v <<= 4;
            if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
            else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
            else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
            else fail("syntax error while parsing value - invalid string: '\\u' must be followed by 4 hex digits");
        }
        return v;
    }

    std::string parse_string() {
        ++pos_;  // opening quote
        std::string out;
        for (;;) {
            if (pos_ >= n_) fail("syntax error while parsing value - invalid string: missing closing quote");
            unsigned char c = (unsigned char)s_[pos_];
            if (c == '"') { ++pos_; return out; }
            if (c < 0x20) fail("syntax error while parsing value - invalid string: control character must be escaped");
            if (c == '\\') {
                ++pos_;
                if (pos_ >= n_) fail("syntax error while parsing value - invalid string: missing closing quote");
                char e = s_[pos_++];
                switch (e) {
                    case '"': out.push_back('"'); break;
                    case '\\': out.push_back('\\'); break;
                    case '/': out.push_back('/'); break;
                    case 'b': out.push_back('\b'); break;
                    case 'f': out.push_back('\f'); break;
                    case 'n': out.push_back('\n'); break;
                    case 'r': out.push_back('\r'); break;
                    case 't': out.push_back('\t'); break;
                    case 'u': {
                        uint32_t cp = parse_hex4();
                        if (cp >= 0xD800 && cp <= 0xDBFF) {
                            if (pos_ + 2 <= n_ && s_[pos_] == '\\' && s_[pos_ + 1] == 'u') {
                                pos_ += 2;
                                uint32_t lo = parse_hex4();
                                if (lo < 0xDC00 || lo > 0xDFFF)
                                    fail("syntax error while parsing value - invalid string: surrogate U+D800..U+DBFF must be followed by U+DC00..U+DFFF");
                                cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                            } else {
                                fail("syntax error while parsing value - invalid string: surrogate U+D800..U+DBFF must be followed by U+DC00..U+DFFF");
                            }
                        } else if (cp >= 0xDC00 && cp <= 0xDFFF) {
                            fail("syntax error while parsing value - invalid string: surrogate U+DC00..U+DFFF must follow U+D800..U+DBFF");
                        }
                        append_utf8(out, cp);
                        break;
                    }
                    default:
                        fail("syntax error while parsing value - invalid string: forbidden character after backslash");
                }
                continue;
            }
            // UTF-8 validation (nlohmann rejects ill-formed sequences).
            size_t len = 0;
            if (c < 0x80) len = 1;
            else if (c >= 0xC2 && c <= 0xDF) len = 2;
            else if (c >= 0xE0 && c <= 0xEF) len = 3;
            else if (c >= 0xF0 && c <= 0xF4) len = 4;
            else fail("syntax error while parsing value - invalid string: ill-formed UTF-8 byte");
            if (pos_ + len > n_) fail("syntax error while parsing value - invalid string: ill-formed UTF-8 byte");
            for (size_t k = 1; k < len; ++k) {
                unsigned char cc = (unsigned char)s_[pos_ + k];
                unsigned lo = 0x80, hi = 0xBF;
                if (k == 1) {
                    if (c == 0xE0) lo = 0xA0;
                    else if (c == 0xED) hi = 0x9F;
                    else if (c == 0xF0) lo = 0x90;
                    else if (c == 0xF4) hi = 0x8F;
                }
                if (cc < lo || cc > hi) fail("syntax error while parsing value - invalid string: ill-formed UTF-8 byte");
            }
            out.append(s_, pos_, len);
            pos_ += len;
        }
    }

    Value parse_number() {
        size_t start = pos_;
        bool neg = false, is_float = false;
        if (s_[pos_] == '-') { neg = true; ++pos_; }
        if (pos_ >= n_) fail("syntax error while parsing value - invalid number; expected digit after '-'");
        if (s_[pos_] == '0') {
            ++pos_;
        } else if (s_[pos_] >= '1' && s_[pos_] <= '9') {
            while (pos_ < n_ && s_[pos_] >= '0' && s_[pos_] <= '9') ++pos_;
        } else {
            fail("syntax error while parsing value - invalid number; expected digit after '-'");
        }
        if (pos_ < n_ && s_[pos_] == '.') {
            is_float = true;
            ++pos_;
            if (pos_ >= n_ || !(s_[pos_] >= '0' && s_[pos_] <= '9'))
                fail("syntax error while parsing value - invalid number; expected digit after '.'");
            while (pos_ < n_ && s_[pos_] >= '0' && s_[pos_] <= '9') ++pos_;
        }
        if (pos_ < n_ && (s_[pos_] == 'e' || s_[pos_] == 'E')) {
            is_float = true;
            ++pos_;
            if (pos_ < n_ && (s_[pos_] == '+' || s_[pos_] == '-')) ++pos_;
            if (pos_ >= n_ || !(s_[pos_] >= '0' && s_[pos_] <= '9'))
                fail("syntax error while parsing value - invalid number; expected digit after exponent sign");
            while (pos_ < n_ && s_[pos_] >= '0' && s_[pos_] <= '9') ++pos_;
        }
        std::string tok = s_.substr(start, pos_ - start);
        Value v;
        if (!is_float) {
            errno = 0;
            char* end = nullptr;
            if (neg) {
                long long x = std::strtoll(tok.c_str(), &end, 10);
                if (errno == 0 && end && *end == '\0') {
                    v.type_ = Value::Type::Integer;
                    v.i_ = x;
                    return v;
                }
            } else {
                unsigned long long x = std::strtoull(tok.c_str(), &end, 10);
                if (errno == 0 && end && *end == '\0') {
                    v.type_ = Value::Type::Unsigned;
                    v.u_ = x;
                    return v;
                }
            }
            // overflow: fall through to a float like nlohmann
        }
        v.type_ = Value::Type::Float;
        v.d_ = strtod_c(tok);
        return v;
    }

    static double strtod_c(const std::string& tok) {
        // The token grammar above never contains locale-dependent characters
        // other than '.', which strtod_l with the C locale handles exactly.
        static locale_t cloc = newlocale(LC_NUMERIC_MASK, "C", (locale_t)0);
        return strtod_l(tok.c_str(), nullptr, cloc);
    }
};

Value Value::parse(const std::string& text) {
    Parser p(text);
    return p.parse_document();
}

}  // namespace rtjson
