// solvempc_amd/cpp/json_lite.hpp — minimal JSON reader for the flat numeric config schema of
// config/MPC_API.json (objects, arrays, numbers, strings, true/false/null).  Replaces the vendored
// nlohmann/json 3.9.1 for this path; errors throw json_lite::error (the reference throws
// nlohmann::detail::parse_error / type_error at ModelPredictiveControlAPI.cpp:13,437,461,471,480).
#pragma once

#include <cctype>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace json_lite {

struct error : std::runtime_error {
    using std::runtime_error::runtime_error;
};

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
    size_t size() const { return kind == Array ? arr.size() : kind == Object ? obj.size() : 1; }
    const Value &operator[](const std::string &k) const
    {
        auto it = obj.find(k);
        if (kind != Object || it == obj.end()) throw error("missing key \"" + k + "\"");
        return it->second;
    }
    bool contains(const std::string &k) const { return kind == Object && obj.count(k); }
    const Value &at(size_t i) const
    {
        if (kind != Array || i >= arr.size()) throw error("index out of range");
        return arr[i];
    }
    double get_double() const
    {
        if (kind != Number) throw error("type_error: expected a number");
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
        if (i_ != s_.size()) throw error("parse_error: trailing characters");
        return v;
    }

private:
    void ws()
    {
        while (i_ < s_.size() && std::isspace((unsigned char)s_[i_])) i_++;
    }
    char peek()
    {
        ws();
        if (i_ >= s_.size()) throw error("parse_error: unexpected end of input");
        return s_[i_];
    }
    void expect(char c)
    {
        if (peek() != c) throw error(std::string("parse_error: expected '") + c + "'");
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
                if (k.kind != Value::String) throw error("parse_error: object key must be a string");
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
            if (i_ >= s_.size()) throw error("parse_error: unterminated string");
            i_++;
            return v;
        }
        if (s_.compare(i_, 4, "true") == 0) { i_ += 4; v.kind = Value::Bool; v.b = true; return v; }
        if (s_.compare(i_, 5, "false") == 0) { i_ += 5; v.kind = Value::Bool; return v; }
        if (s_.compare(i_, 4, "null") == 0) { i_ += 4; return v; }
        const char *b = s_.c_str() + i_;
        char *e = nullptr;
        const double d = std::strtod(b, &e);
        if (e == b) throw error("parse_error: invalid literal");
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
