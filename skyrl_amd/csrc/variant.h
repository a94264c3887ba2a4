// Kernel variant knobs (see variant.hip): every kernel family reads its A/B choices through
// knobs(), which is the tuned defaults except while a *_ex call with a variant runs.
#pragma once
#include "common.h"

namespace skyrl {

struct Knobs {
    int logprob_unroll = 4;
    int logprob_nt = 1;
    int train_resident = 1;
    int train_resident_nt = 1024;
    int train_ntstore = 1;
    int train_split = 1;
    int train_split_shape = 0;
    int train_split_wait = 5000;  // ticks of the 100 MHz constant clock: 50 us
    int grpo_slices = 4;
    int loss_units = 0;
    int loss_bwd_blocks = 256;
    int grpo_loss_rpb = 1;
    int finish_mode = 0;
    int sampler_row = 1;
    int sampler_split_rows = 256;
    int sampler_split_wgs = 1024;
    int sampler_split_nt = 256;
    int sampler_split_gran = 8192;
    int sampler_topk_fast = 1;
    int sampler_topp_fast = 1;
    int topp_probe = 0;
    int lmhead_pipe = 12;
    int lmhead_group = 8;
    int attn_pf = 0;
    int lmhead_persist = 4;
};
inline constexpr Knobs kDefaultKnobs{};

// the variant of the running call (the defaults outside *_ex calls); header-inline so that a
// probe build of one kernel file links without variant.hip
namespace detail {
inline thread_local const Knobs* tl_knobs = nullptr;
}  // namespace detail
inline const Knobs& knobs() { return detail::tl_knobs ? *detail::tl_knobs : kDefaultKnobs; }

// installs a validated variant for the lifetime of one *_ex call
class VariantScope {
  public:
    VariantScope() = default;
    VariantScope(const VariantScope&) = delete;
    VariantScope& operator=(const VariantScope&) = delete;
    int enter(const skyrl_variant* v);
    ~VariantScope();

  private:
    Knobs k_;
    const Knobs* prev_ = nullptr;
    bool active_ = false;
};

}  // namespace skyrl
