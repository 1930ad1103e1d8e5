// model_library.hpp -- internal: the C-ABI entry points of the library serving a model (libmmpc.so for the
// built-in models, <name>.so for a model generated from SX).  Shared by ModelControl and BatchModelControl.
#pragma once
#include <dlfcn.h>

#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include <Mahi/Mpc/ModelParameters.hpp>

#include "../../../include/mmpc.h"

namespace mahi {
namespace mpc {
namespace detail {

// The solver entry points of the model's library.  The reference loads the model's compiled NLP from the JSON's
// dll_filepath (ModelControl.cpp:62, nlpsol over <name>.so); here a model generated from SX dynamics has its own
// <name>.so exporting the C-ABI of include/mmpc.h (ModelGenerator::compile_model), and the built-in models are
// served by the linked libmmpc.so.
struct ModelLibrary {
    decltype(&mmpc_create_from_json) create_from_json = &mmpc_create_from_json;
    decltype(&mmpc_destroy) destroy = &mmpc_destroy;
    decltype(&mmpc_get_model_info) get_model_info = &mmpc_get_model_info;
    decltype(&mmpc_solve_batch_host) solve_batch_host = &mmpc_solve_batch_host;
    decltype(&mmpc_solve_batch) solve_batch = &mmpc_solve_batch;
    decltype(&mmpc_reserve_workspace) reserve_workspace = &mmpc_reserve_workspace;
    decltype(&mmpc_last_error) last_error = &mmpc_last_error;
    void* dl = nullptr;  // kept loaded for the process lifetime (HIP code objects), as CasADi keeps its libraries

    void check(int rc, const char* what) const {
        if (rc != MMPC_OK) throw std::runtime_error(std::string(what) + ": " + last_error());
    }
    template <class F>
    void bind(F& f, const char* name) {
        void* s = dlsym(dl, name);
        if (!s) throw std::runtime_error(std::string("model library lacks ") + name);
        f = reinterpret_cast<F>(s);
    }
    // dll_filepath relative to the JSON's directory first, then to the working directory
    // A generated model names itself in "mmpc_model"; built-in models (and reference-written JSONs, whose
    // dll_filepath is a CasADi NLP library) are served by libmmpc.so.
    static std::shared_ptr<ModelLibrary> load(const ModelParameters& mp, const std::string& json_path) {
        auto b = std::make_shared<ModelLibrary>();
        const std::string& dll = mp.dll_filepath;
        const size_t sl = dll.rfind('/');
        const std::string base = sl == std::string::npos ? dll : dll.substr(sl + 1);
        const std::string& mm = mp.mmpc_model;
        if (mm.empty() || mm == "two_link_arm" || mm == "double_pendulum" || mm == "exo_arm" || mm == "exo" ||
            dll.empty() || base == "libmmpc.so")
            return b;
        std::vector<std::string> cands;
        if (dll[0] != '/') {
            const size_t js = json_path.rfind('/');
            if (js != std::string::npos) cands.push_back(json_path.substr(0, js + 1) + dll);
        }
        cands.push_back(dll[0] == '/' || dll.find('/') != std::string::npos ? dll : "./" + dll);
        std::string errs;
        for (const std::string& c : cands) {
            b->dl = dlopen(c.c_str(), RTLD_NOW | RTLD_LOCAL);
            if (b->dl) break;
            const char* e = dlerror();
            errs += std::string("\n  ") + c + ": " + (e ? e : "?");
        }
        if (!b->dl) throw std::runtime_error("cannot load the model library " + dll + errs);
        b->bind(b->create_from_json, "mmpc_create_from_json");
        b->bind(b->destroy, "mmpc_destroy");
        b->bind(b->get_model_info, "mmpc_get_model_info");
        b->bind(b->solve_batch_host, "mmpc_solve_batch_host");
        b->bind(b->solve_batch, "mmpc_solve_batch");
        b->bind(b->reserve_workspace, "mmpc_reserve_workspace");
        b->bind(b->last_error, "mmpc_last_error");
        return b;
    }
};

}  // namespace detail
}  // namespace mpc
}  // namespace mahi
