// knobs.h -- tuning and diagnostic overrides of libsiddhi_hip.so (kernel A/B experiments, traces,
// test hooks that force a code path). The library reads no environment variables: every knob comes
// from sdh_config.debug, "NAME=VALUE;NAME=VALUE" (include/siddhi_hip.h), parsed at engine creation.
// sdh::knob(name) sees the knobs of the engine whose ABI call is running on this thread (nullptr:
// unset, or no engine -- e.g. sdh_spec_selftest). DESIGN.md §8 lists the names.
#pragma once

namespace sdh {
const char* knob(const char* name);
}
