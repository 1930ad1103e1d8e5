// json_lite.h -- minimal JSON reader for the <name>.json model file.
//
// The reference serialises ModelParameters with nlohmann::json through mahi-util
// (src/Mahi/Mpc/ModelParameters.cpp:37-50, written by ModelGenerator::save_param_file,
// ModelGenerator.cpp:261-270).  Neither library is available here, so this is a small
// recursive-descent reader for exactly the value kinds that file uses
// (objects, arrays, numbers, strings, booleans, null).
#pragma once
#include <cctype>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace mmpc {
namespace json {

struct Value {
    enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
    bool b = false;
    double num = 0.0;
    std::string str;
    std::vector<Value> arr;
    std::map<std::string, Value> obj;

    const Value* get(const std::string& k) const {
        if (kind != Object) return nullptr;
        auto it = obj.find(k);
        return it == obj.end() ? nullptr : &it->second;
    }
};

class Parser {
public:
    explicit Parser(const std::string& s) : s_(s) {}
    Value parse() {
        Value v = value();
        ws();
        if (i_ != s_.size()) fail("trailing characters");
        return v;
    }

private:
    const std::string& s_;
    size_t i_ = 0;
    int depth_ = 0;  // nesting of the value being parsed (recursive descent: bounded so input cannot overflow the stack)
    static constexpr int kMaxDepth = 64;

    [[noreturn]] void fail(const char* what) {
        throw std::runtime_error(std::string("json: ") + what + " at offset " + std::to_string(i_));
    }
    void ws() {
        while (i_ < s_.size() && std::isspace(static_cast<unsigned char>(s_[i_]))) ++i_;
    }
    bool lit(const char* w) {
        size_t n = std::char_traits<char>::length(w);
        if (s_.compare(i_, n, w) == 0) {
            i_ += n;
            return true;
        }
        return false;
    }
    struct DepthGuard {
        int& d;
        explicit DepthGuard(int& d_) : d(d_) { ++d; }
        ~DepthGuard() { --d; }
    };
    Value value() {
        DepthGuard guard(depth_);
        if (depth_ > kMaxDepth) fail("nesting too deep");
        ws();
        if (i_ >= s_.size()) fail("unexpected end");
        char c = s_[i_];
        Value v;
        if (c == '{') {
            v.kind = Value::Object;
            ++i_;
            ws();
            if (i_ < s_.size() && s_[i_] == '}') {
                ++i_;
                return v;
            }
            for (;;) {
                ws();
                if (i_ >= s_.size() || s_[i_] != '"') fail("expected key");
                std::string k = string();
                ws();
                if (i_ >= s_.size() || s_[i_] != ':') fail("expected ':'");
                ++i_;
                v.obj[k] = value();
                ws();
                if (i_ < s_.size() && s_[i_] == ',') {
                    ++i_;
                    continue;
                }
                if (i_ < s_.size() && s_[i_] == '}') {
                    ++i_;
                    break;
                }
                fail("expected ',' or '}'");
            }
        } else if (c == '[') {
            v.kind = Value::Array;
            ++i_;
            ws();
            if (i_ < s_.size() && s_[i_] == ']') {
                ++i_;
                return v;
            }
            for (;;) {
                v.arr.push_back(value());
                ws();
                if (i_ < s_.size() && s_[i_] == ',') {
                    ++i_;
                    continue;
                }
                if (i_ < s_.size() && s_[i_] == ']') {
                    ++i_;
                    break;
                }
                fail("expected ',' or ']'");
            }
        } else if (c == '"') {
            v.kind = Value::String;
            v.str = string();
        } else if (lit("true")) {
            v.kind = Value::Bool;
            v.b = true;
        } else if (lit("false")) {
            v.kind = Value::Bool;
            v.b = false;
        } else if (lit("null")) {
            v.kind = Value::Null;
        } else {
            const char* start = s_.c_str() + i_;
            char* end = nullptr;
            v.num = std::strtod(start, &end);
            if (end == start) fail("bad value");
            v.kind = Value::Number;
            i_ += static_cast<size_t>(end - start);
        }
        return v;
    }
    std::string string() {
        ++i_;  // opening quote
        std::string out;
        while (i_ < s_.size() && s_[i_] != '"') {
            char c = s_[i_++];
            if (c == '\\') {
                if (i_ >= s_.size()) fail("bad escape");
                char e = s_[i_++];
                switch (e) {
                    case 'n': out += '\n'; break;
                    case 't': out += '\t'; break;
                    case 'r': out += '\r'; break;
                    case 'b': out += '\b'; break;
                    case 'f': out += '\f'; break;
                    case 'u': {
                        if (i_ + 4 > s_.size()) fail("bad \\u");
                        unsigned cp = std::strtoul(s_.substr(i_, 4).c_str(), nullptr, 16);
                        i_ += 4;
                        if (cp < 0x80) out += static_cast<char>(cp);
                        else out += '?';
                        break;
                    }
                    default: out += e;
                }
            } else {
                out += c;
            }
        }
        if (i_ >= s_.size()) fail("unterminated string");
        ++i_;
        return out;
    }
};

inline Value parse(const std::string& s) { return Parser(s).parse(); }

}  // namespace json
}  // namespace mmpc
