// Host-side RAII wrappers over the C ABI (include/addapt_gpu.h).  Internal to
// the host library.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "addapt_gpu.h"

namespace addapt {
namespace gpu {

inline void check(adx_status s) {
    if (s != ADX_OK) throw std::string(adx_last_error());
}

/// process-wide parameter set (addapt_amd/data/rna_turner2004_addapt.par by default,
/// ADX_PARAMS or set_parameter_file() to override)
const adx_params *params();
void set_params_path(const std::string &path);

struct FoldDel {
    void operator()(adx_fold *f) const { adx_fold_free(f); }
};
using FoldPtr = std::unique_ptr<adx_fold, FoldDel>;

struct CtxDel {
    void operator()(adx_ctx *c) const { adx_ctx_destroy(c); }
};
using CtxPtr = std::unique_ptr<adx_ctx, CtxDel>;

}  // namespace gpu
}  // namespace addapt
