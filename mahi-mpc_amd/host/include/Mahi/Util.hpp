// Mahi/Util.hpp -- the subset of mahi-util (a third-party dependency of the reference, FetchContent in its
// CMakeLists.txt:42; not in this image) that the reference's built examples use, so that
// examples/ex_model_generate.cpp, model_control_example.cpp and thread_model_control_example.cpp compile unchanged
// against this mirror: PI, Time / seconds / milliseconds, Clock, Timestamp, print with {} and {:.Nf} fields,
// Options (the cxxopts-style add_options / parse / count used at model_control_example.cpp:10-16), sleep and the
// realtime toggles, Timer.  Behaviour follows mahi-util's documented semantics for these calls; nothing else is provided.
#pragma once
#include <Mahi/Util/Time.hpp>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <ctime>
#include <fstream>
#include <iostream>
#include <map>
#include <set>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

namespace mahi {
namespace util {

constexpr double PI = 3.14159265358979323846;

// Time / Time is a ratio (mahi-util semantics: sim_time / time_step = number of steps)
inline double operator/(const Time& a, const Time& b) {
    return static_cast<double>(a.as_microseconds()) / static_cast<double>(b.as_microseconds());
}
inline std::ostream& operator<<(std::ostream& os, const Time& t) { return os << t.as_seconds() << " s"; }

// wall clock since construction or the last restart()
class Clock {
public:
    Clock() : t0_(std::chrono::steady_clock::now()) {}
    Time get_elapsed_time() const {
        return microseconds(std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0_)
                                .count());
    }
    Time restart() {
        const Time e = get_elapsed_time();
        t0_ = std::chrono::steady_clock::now();
        return e;
    }

private:
    std::chrono::steady_clock::time_point t0_;
};

// fixed-rate loop timer: wait() sleeps until the next multiple of the period since construction and returns the
// elapsed time (mahi::util::Timer(Time period); the reference's thread example paces its plant with it)
class Timer {
public:
    explicit Timer(Time period) : period_us_(period.as_microseconds() > 0 ? period.as_microseconds() : 1) {}
    Time wait() {
        ++ticks_;
        const auto target = clock_start_ + std::chrono::microseconds(ticks_ * period_us_);
        if (std::chrono::steady_clock::now() < target) std::this_thread::sleep_until(target);
        return get_elapsed_time();
    }
    Time get_elapsed_time() const {
        return microseconds(
            std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - clock_start_).count());
    }
    Time get_period() const { return microseconds(period_us_); }
    Time restart() {
        const Time e = get_elapsed_time();
        clock_start_ = std::chrono::steady_clock::now();
        ticks_ = 0;
        return e;
    }

private:
    int64_t period_us_;
    int64_t ticks_ = 0;
    std::chrono::steady_clock::time_point clock_start_ = std::chrono::steady_clock::now();
};

inline void sleep(Time t) { std::this_thread::sleep_for(std::chrono::microseconds(t.as_microseconds())); }
// process priority toggles: no-ops here (the solve runs on the GPU; the reference raises the Windows/Linux
// scheduling class, which needs privileges the controller host may not grant)
inline bool enable_realtime() { return true; }
inline bool disable_realtime() { return true; }

// local wall-clock time stamp taken at construction
class Timestamp {
public:
    Timestamp() {
        const auto now = std::chrono::system_clock::now();
        const std::time_t t = std::chrono::system_clock::to_time_t(now);
        ms_ = static_cast<int>(
            std::chrono::duration_cast<std::chrono::milliseconds>(now.time_since_epoch()).count() % 1000);
        localtime_r(&t, &tm_);
    }
    std::string yyyy_mm_dd() const { return fmt("%04d-%02d-%02d", tm_.tm_year + 1900, tm_.tm_mon + 1, tm_.tm_mday); }
    std::string hh_mm_ss() const { return fmt("%02d:%02d:%02d", tm_.tm_hour, tm_.tm_min, tm_.tm_sec); }
    std::string hh_mm_ss_mmm() const { return hh_mm_ss() + fmt(".%03d", ms_); }
    std::string yyyy_mm_dd_hh_mm_ss() const { return yyyy_mm_dd() + "_" + fmt("%02d.%02d.%02d", tm_.tm_hour, tm_.tm_min, tm_.tm_sec); }

private:
    template <class... A>
    static std::string fmt(const char* f, A... a) {
        char buf[64];
        std::snprintf(buf, sizeof buf, f, a...);
        return buf;
    }
    std::tm tm_{};
    int ms_ = 0;
};

namespace detail {
// one replacement field: "" (default formatting) or ".Nf" / ".Ne" / ".Ng" (precision + presentation)
template <class T>
void format_field(std::ostringstream& os, const std::string& spec, const T& v) {
    std::ostringstream f;
    if (!spec.empty()) {
        if (spec.size() < 3 || spec[0] != '.') throw std::invalid_argument("mahi::util::print: unsupported field {:" + spec + "}");
        const int prec = std::stoi(spec.substr(1, spec.size() - 2));
        const char ty = spec.back();
        f.precision(prec);
        if (ty == 'f') f << std::fixed;
        else if (ty == 'e') f << std::scientific;
        else if (ty != 'g') throw std::invalid_argument("mahi::util::print: unsupported field {:" + spec + "}");
    }
    f << v;
    os << f.str();
}
inline void format_rest(std::ostringstream& os, const std::string& s, size_t i) {
    for (; i < s.size(); ++i) {
        if ((s[i] == '{' || s[i] == '}') && i + 1 < s.size() && s[i + 1] == s[i]) ++i;   // {{ and }}
        else if (s[i] == '{') throw std::invalid_argument("mahi::util::print: more fields than arguments");
        os << s[i];
    }
}
template <class T, class... R>
void format_rest(std::ostringstream& os, const std::string& s, size_t i, const T& v, const R&... rest) {
    for (; i < s.size(); ++i) {
        if ((s[i] == '{' || s[i] == '}') && i + 1 < s.size() && s[i + 1] == s[i]) {
            os << s[i++];
        } else if (s[i] == '{') {
            const size_t e = s.find('}', i);
            if (e == std::string::npos) throw std::invalid_argument("mahi::util::print: unterminated field");
            std::string spec = s.substr(i + 1, e - i - 1);
            if (!spec.empty() && spec[0] == ':') spec = spec.substr(1);
            format_field(os, spec, v);
            format_rest(os, s, e + 1, rest...);
            return;
        } else {
            os << s[i];
        }
    }
}
}  // namespace detail

// fmt-style formatting of the subset used by the reference's examples ({} and {:.2f})
template <class... A>
std::string format(const std::string& f, const A&... a) {
    std::ostringstream os;
    detail::format_rest(os, f, 0, a...);
    return os.str();
}
template <class... A>
void print(const std::string& f, const A&... a) {
    std::cout << format(f, a...) << std::endl;
}

// command-line options, the cxxopts subset: add_options()("s,long", "help"[, value]) and parse(argc, argv) whose
// result answers count("long") / count("s") and operator[]("long").as<T>()
template <class T>
struct ValueType {};
// value<T>(): the third argument of add_options()(...) for options that take a value (cxxopts::value<T>())
template <class T>
ValueType<T> value() {
    return {};
}

namespace detail {
template <class T>
struct OptionParse {
    static T get(const std::string& text) {
        std::istringstream is(text);
        T v{};
        if (!(is >> v)) throw std::invalid_argument("bad option value: " + text);
        return v;
    }
};
template <>
struct OptionParse<std::string> {
    static std::string get(const std::string& text) { return text; }
};
template <class T>
struct OptionParse<std::vector<T>> {   // comma-separated list, as cxxopts
    static std::vector<T> get(const std::string& text) {
        std::vector<T> out;
        std::string item;
        std::istringstream is(text);
        while (std::getline(is, item, ',')) out.push_back(OptionParse<T>::get(item));
        return out;
    }
};
}  // namespace detail

class Options {
public:
    struct Value {
        std::string text;
        template <class T>
        T as() const {
            return detail::OptionParse<T>::get(text);
        }
    };
    class Result {
    public:
        size_t count(const std::string& name) const { return seen_.count(name); }
        Value operator[](const std::string& name) const {
            auto it = values_.find(name);
            if (it == values_.end()) throw std::out_of_range("option not given: " + name);
            return Value{it->second};
        }
        const std::vector<std::string>& unmatched() const { return unmatched_; }

    private:
        friend class Options;
        std::set<std::string> seen_;
        std::map<std::string, std::string> values_;
        std::vector<std::string> unmatched_;
    };
    struct Adder {
        Options* o;
        Adder& operator()(const std::string& names, const std::string& help) {
            o->add(names, help, false);
            return *this;
        }
        template <class T>
        Adder& operator()(const std::string& names, const std::string& help, ValueType<T>) {
            o->add(names, help, true);
            return *this;
        }
    };
    Options(std::string program, std::string description) : program_(std::move(program)), desc_(std::move(description)) {}
    Adder add_options() { return Adder{this}; }
    Result parse(int argc, char* argv[]) const {
        Result r;
        for (int i = 1; i < argc; ++i) {
            std::string a = argv[i], val;
            bool has_val = false;
            if (a.rfind("--", 0) == 0) {
                a = a.substr(2);
            } else if (a.size() >= 2 && a[0] == '-') {
                a = a.substr(1);
            } else {
                r.unmatched_.push_back(a);
                continue;
            }
            const size_t eq = a.find('=');
            if (eq != std::string::npos) {
                val = a.substr(eq + 1);
                a = a.substr(0, eq);
                has_val = true;
            }
            auto it = alias_.find(a);
            if (it == alias_.end()) throw std::invalid_argument("unknown option: " + a);
            const Opt& o = opts_[it->second];
            if (o.takes_value && !has_val) {
                if (i + 1 >= argc) throw std::invalid_argument("option needs a value: " + a);
                val = argv[++i];
            }
            r.seen_.insert(o.shrt);
            r.seen_.insert(o.lng);
            if (o.takes_value) {
                r.values_[o.shrt] = val;
                r.values_[o.lng] = val;
            }
        }
        return r;
    }
    std::string help() const {
        std::ostringstream os;
        os << desc_ << "\nUsage: " << program_ << " [OPTION...]\n";
        for (const Opt& o : opts_) os << "  " << (o.shrt.empty() ? "   " : "-" + o.shrt + ",") << " --" << o.lng << "  " << o.help << "\n";
        return os.str();
    }

private:
    struct Opt {
        std::string shrt, lng, help;
        bool takes_value;
    };
    void add(const std::string& names, const std::string& help, bool takes_value) {
        Opt o;
        const size_t c = names.find(',');
        if (c == std::string::npos) {
            o.lng = trim(names);
        } else {
            o.shrt = trim(names.substr(0, c));
            o.lng = trim(names.substr(c + 1));
        }
        o.help = help;
        o.takes_value = takes_value;
        const size_t idx = opts_.size();
        opts_.push_back(o);
        if (!o.shrt.empty()) alias_[o.shrt] = idx;
        alias_[o.lng] = idx;
    }
    static std::string trim(const std::string& t) {
        const size_t b = t.find_first_not_of(' '), e = t.find_last_not_of(' ');
        return b == std::string::npos ? std::string() : t.substr(b, e - b + 1);
    }
    std::string program_, desc_;
    std::vector<Opt> opts_;
    std::map<std::string, size_t> alias_;
};

}  // namespace util
}  // namespace mahi
