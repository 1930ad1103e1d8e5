// Mahi/Util/Time.hpp -- the subset of mahi::util::Time used by the mahi-mpc public headers
// (ModelControl.hpp:17,32,35,40; ModelParameters.hpp:12,17-18): an int64 microsecond count.
#pragma once
#include <cstdint>

namespace mahi {
namespace util {

class Time {
public:
    constexpr Time() : us_(0) {}
    static constexpr Time from_us(int64_t us) { return Time(us); }
    constexpr double as_seconds() const { return static_cast<double>(us_) * 1e-6; }
    constexpr double as_milliseconds() const { return static_cast<double>(us_) * 1e-3; }
    constexpr int64_t as_microseconds() const { return us_; }
    constexpr bool operator<(const Time& o) const { return us_ < o.us_; }
    constexpr bool operator>(const Time& o) const { return us_ > o.us_; }
    constexpr bool operator<=(const Time& o) const { return us_ <= o.us_; }
    constexpr bool operator>=(const Time& o) const { return us_ >= o.us_; }
    constexpr bool operator==(const Time& o) const { return us_ == o.us_; }
    constexpr bool operator!=(const Time& o) const { return us_ != o.us_; }
    constexpr Time operator+(const Time& o) const { return Time(us_ + o.us_); }
    constexpr Time operator-(const Time& o) const { return Time(us_ - o.us_); }

private:
    explicit constexpr Time(int64_t us) : us_(us) {}
    int64_t us_;
};

inline Time seconds(double s) { return Time::from_us(static_cast<int64_t>(s * 1e6 + (s >= 0 ? 0.5 : -0.5))); }
inline Time milliseconds(double ms) { return Time::from_us(static_cast<int64_t>(ms * 1e3 + (ms >= 0 ? 0.5 : -0.5))); }
inline Time microseconds(int64_t us) { return Time::from_us(us); }

}  // namespace util
}  // namespace mahi
