// solvempc_amd/cpp/json_lite.hpp — minimal JSON reader for the flat numeric config schema of
// config/MPC_API.json (objects, arrays, numbers, strings, true/false/null).  Replaces the vendored
// nlohmann/json 3.9.1 for this path.  Errors keep nlohmann's observable shape: a
// json_lite::detail::exception hierarchy (parse_error, type_error, out_of_range) with an integer `id`
// and what() = "[json.exception.<kind>.<id>] <message>", thrown where the reference's json throws
// (json::parse of a missing/garbled file, ModelPredictiveControlAPI.cpp:12-13: parse_error 101;
// get<double>() of a non-number, :19: type_error 302; from_json's own throws, :437,461,471,480:
// type_error::create(0, "")).
#pragma once

#include <cctype>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace json_lite {

namespace detail {
class exception : public std::exception {
public:
    const int id;
    const char *what() const noexcept override { return m_.what(); }

protected:
    exception(int id_, const std::string &kind, const std::string &msg)
        : id(id_), m_("[json.exception." + kind + "." + std::to_string(id_) + "] " + msg) {}

private:
    std::runtime_error m_;
};
class parse_error : public exception {
public:
    static parse_error create(int id_, std::size_t byte_, const std::string &msg)
    {
        return parse_error(id_, byte_, "parse error at byte " + std::to_string(byte_) + ": " + msg);
    }
    const std::size_t byte;

private:
    parse_error(int id_, std::size_t byte_, const std::string &msg) : exception(id_, "parse_error", msg), byte(byte_) {}
};
class type_error : public exception {
public:
    static type_error create(int id_, const std::string &msg) { return type_error(id_, msg); }

private:
    type_error(int id_, const std::string &msg) : exception(id_, "type_error", msg) {}
};
class out_of_range : public exception {
public:
    static out_of_range create(int id_, const std::string &msg) { return out_of_range(id_, msg); }

private:
    out_of_range(int id_, const std::string &msg) : exception(id_, "out_of_range", msg) {}
};
}  // namespace detail
using error = detail::exception;  // the base every json_lite error derives from

struct Value {
    enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
    double num = 0.0;
    bool b = false;
    std::string str;
    std::vector<Value> arr;
    std::map<std::string, Value> obj;

    bool is_number() const { return kind == Number; }
    bool is_array() const { return kind == Array; }
    bool empty() const { return kind == Array ? arr.empty() : kind == Object ? obj.empty() : kind == Null; }
    size_t size() const { return kind == Array ? arr.size() : kind == Object ? obj.size() : kind == Null ? 0 : 1; }
    // A missing key reads as null (nlohmann's non-const operator[] inserts one), so the caller's
    // conversion throws the type_error the reference's would.
    const Value &operator[](const std::string &k) const
    {
        static const Value null_value;
        if (kind != Object) throw detail::type_error::create(305, "cannot use operator[] with a string argument with " + type_name());
        auto it = obj.find(k);
        return it == obj.end() ? null_value : it->second;
    }
    std::string type_name() const
    {
        static const char *names[] = {"null", "boolean", "number", "string", "array", "object"};
        return names[kind];
    }
    bool contains(const std::string &k) const { return kind == Object && obj.count(k); }
    const Value &at(size_t i) const
    {
        if (kind != Array) throw detail::type_error::create(304, "cannot use at() with " + type_name());
        if (i >= arr.size()) throw detail::out_of_range::create(401, "array index " + std::to_string(i) + " is out of range");
        return arr[i];
    }
    double get_double() const
    {
        if (kind != Number) throw detail::type_error::create(302, "type must be number, but is " + type_name());
        return num;
    }
};

class Parser {
public:
    explicit Parser(const std::string &s) : s_(s) {}
    Value parse()
    {
        Value v = value();
        ws();
        if (i_ != s_.size()) throw bad("syntax error: trailing characters");
        return v;
    }

private:
    detail::parse_error bad(const std::string &msg) const { return detail::parse_error::create(101, i_ + 1, msg); }
    void ws()
    {
        while (i_ < s_.size() && std::isspace((unsigned char)s_[i_])) i_++;
    }
    char peek()
    {
        ws();
        if (i_ >= s_.size()) throw bad("syntax error: unexpected end of input");
        return s_[i_];
    }
    void expect(char c)
    {
        if (peek() != c) throw bad(std::string("syntax error: expected '") + c + "'");
        i_++;
    }
    Value value()
    {
        const char c = peek();
        Value v;
        if (c == '{') {
            v.kind = Value::Object;
            i_++;
            if (peek() == '}') { i_++; return v; }
            for (;;) {
                Value k = value();
                if (k.kind != Value::String) throw bad("syntax error: object key must be a string");
                expect(':');
                v.obj[k.str] = value();
                if (peek() == ',') { i_++; continue; }
                expect('}');
                return v;
            }
        }
        if (c == '[') {
            v.kind = Value::Array;
            i_++;
            if (peek() == ']') { i_++; return v; }
            for (;;) {
                v.arr.push_back(value());
                if (peek() == ',') { i_++; continue; }
                expect(']');
                return v;
            }
        }
        if (c == '"') {
            v.kind = Value::String;
            i_++;
            while (i_ < s_.size() && s_[i_] != '"') {
                if (s_[i_] == '\\' && i_ + 1 < s_.size()) i_++;
                v.str.push_back(s_[i_++]);
            }
            if (i_ >= s_.size()) throw bad("syntax error: unterminated string");
            i_++;
            return v;
        }
        if (s_.compare(i_, 4, "true") == 0) { i_ += 4; v.kind = Value::Bool; v.b = true; return v; }
        if (s_.compare(i_, 5, "false") == 0) { i_ += 5; v.kind = Value::Bool; return v; }
        if (s_.compare(i_, 4, "null") == 0) { i_ += 4; return v; }
        const char *b = s_.c_str() + i_;
        char *e = nullptr;
        const double d = std::strtod(b, &e);
        if (e == b) throw bad("syntax error: invalid literal");
        i_ += (size_t)(e - b);
        v.kind = Value::Number;
        v.num = d;
        return v;
    }
    const std::string &s_;
    size_t i_ = 0;
};

inline Value parse(const std::string &text) { return Parser(text).parse(); }

}  // namespace json_lite
