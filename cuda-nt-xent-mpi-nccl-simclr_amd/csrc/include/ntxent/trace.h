// ntxent-mi355x — observability and failure-injection hooks of the native runtime.
//
// Tracing: roctx ranges (rocprofiler-sdk-roctx) around every runtime stage, visible in a
// `rocprofv3 --marker-trace` timeline next to the kernels. The reference only has an unused
// ENABLE_PROFILING compile flag (CMakeLists.txt:10,82-84); here ranges are always compiled in
// and switched at run time with NTXENT_ROCTX=1 (or the ENABLE_PROFILING CMake option, which
// flips the default), so a production build pays one predictable branch per stage.
//
// Fault injection (test-only): NTXENT_FAULT=<site>[,<site>...] makes the named site throw
// ntxent::InjectedFault, so error paths (collective failure, bad launch, non-finite loss)
// can be exercised without breaking hardware. Sites: prep, fwd, lse, coef, dz, norm_bwd,
// allgather, allreduce, graph, nonfinite.
#pragma once

#include <stdexcept>
#include <string>

namespace ntxent {

struct InjectedFault : std::runtime_error {
  explicit InjectedFault(const std::string& site) : std::runtime_error("ntxent: injected fault at " + site) {}
};

bool trace_enabled();
void trace_push(const char* name);
void trace_pop();
void trace_mark(const char* name);

// Throws InjectedFault if `site` is listed in NTXENT_FAULT (parsed once; override with
// set_fault_sites for in-process tests).
void fault_point(const char* site);
bool fault_armed(const char* site);
void set_fault_sites(const std::string& csv);

class TraceRange {
 public:
  explicit TraceRange(const char* name) : on_(trace_enabled()) {
    if (on_) trace_push(name);
  }
  ~TraceRange() {
    if (on_) trace_pop();
  }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;

 private:
  bool on_;
};

}  // namespace ntxent

#define NTXENT_TRACE_CAT2(a, b) a##b
#define NTXENT_TRACE_CAT(a, b) NTXENT_TRACE_CAT2(a, b)
#define NTXENT_TRACE(name) ::ntxent::TraceRange NTXENT_TRACE_CAT(_ntxent_tr_, __LINE__)(name)
