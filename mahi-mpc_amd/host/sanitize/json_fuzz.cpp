// Sanitizer driver (ASan + UBSan build, `make -C mahi-mpc_amd/host sanitize`): the host-side parsers that read
// user files -- json_lite (csrc/json_lite.h, also compiled into libmmpc) through
// model_parameters_from_json_string (the <name>.json schema of ModelParameters.cpp:37-72) -- on valid, truncated,
// deeply nested and byte-mutated inputs.  Every input must either parse or throw a std::exception; the sanitizers
// turn any out-of-bounds access, leak or undefined behaviour into a non-zero exit.
#include <Mahi/Mpc/ModelParameters.hpp>

#include <cstdint>
#include <cstdio>
#include <exception>
#include <string>
#include <vector>

#include "../../csrc/json_lite.h"

using namespace mahi::mpc;

static int parsed = 0, rejected = 0;

static void feed(const std::string& text) {
    try {
        (void)mmpc::json::parse(text);
        ModelParameters p = model_parameters_from_json_string(text);
        (void)to_json_string(p);
        ++parsed;
    } catch (const std::exception&) {
        ++rejected;
    }
}

int main() {
    const std::string valid =
        "{\"model\": {\"name\": \"double_pendulum\", \"timespan\": 50000, \"step_size\": 2000, \"num_x\": 4, "
        "\"num_u\": 2, \"num_shooting_nodes\": 25, \"x_min\": [-1e31, -1e31, -1e31, -1e31], \"u_min\": [-10, -10], "
        "\"x_max\": [1e31, 1e31, 1e31, 1e31], \"u_max\": [10, 10], \"dll_filepath\": \"double_pendulum.so\", "
        "\"is_linear\": false, \"note\": \"\\u00e9\\n\\t\\\"x\\\"\"}}";
    feed(valid);
    if (parsed != 1) {
        std::fprintf(stderr, "valid model JSON rejected\n");
        return 1;
    }
    for (size_t n = 0; n < valid.size(); ++n) feed(valid.substr(0, n));  // every truncation
    for (int d : {10, 63, 64, 65, 1000, 100000}) {                       // nesting depth
        feed(std::string(static_cast<size_t>(d), '[') + std::string(static_cast<size_t>(d), ']'));
        std::string o;
        for (int i = 0; i < d; ++i) o += "{\"a\":";
        feed(o + "1" + std::string(static_cast<size_t>(d), '}'));
    }
    for (const char* s : {"", " ", "{", "}", "[1,]", "{\"a\"}", "\"\\u12", "\"abc", "nul", "tru", "-", "1e", "1e999",
                          "{\"model\": {\"num_x\": -3}}", "{\"model\": {\"num_x\": 1e300, \"num_u\": 2}}",
                          "{\"model\": {\"x_min\": [1, 2, \"a\"]}}", "{\"model\": []}", "[\"\\", "{\"\\u0000\": 1}"})
        feed(s);
    uint64_t z = 0x9E3779B97F4A7C15ull;  // deterministic byte mutations
    auto next = [&]() {
        z ^= z << 13;
        z ^= z >> 7;
        z ^= z << 17;
        return z;
    };
    for (int t = 0; t < 20000; ++t) {
        std::string m = valid;
        const int edits = 1 + static_cast<int>(next() % 4);
        for (int e = 0; e < edits; ++e) {
            const size_t at = next() % m.size();
            switch (next() % 3) {
                case 0: m[at] = static_cast<char>(next() & 0xff); break;
                case 1: m.erase(at, 1 + next() % 8); break;
                default: m.insert(at, 1, "{}[],:\"\\0123456789eE+-."[next() % 24]);
            }
            if (m.empty()) m = "{";
        }
        feed(m);
    }
    std::printf("json_fuzz ok: %d parsed, %d rejected\n", parsed, rejected);
    return 0;
}
