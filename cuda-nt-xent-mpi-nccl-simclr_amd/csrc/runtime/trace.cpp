// roctx tracing + fault-injection switches (see include/ntxent/trace.h).
#include "ntxent/trace.h"

#include <dlfcn.h>

#include <cstdint>
#include <cstdlib>
#include <mutex>
#include <set>
#include <sstream>

namespace ntxent {
namespace {

bool env_flag(const char* name, bool dflt) {
  const char* e = std::getenv(name);
  if (!e || !*e) return dflt;
  return !(e[0] == '0' || e[0] == 'f' || e[0] == 'F' || e[0] == 'n' || e[0] == 'N');
}

#ifdef NTXENT_PROFILING_DEFAULT
constexpr bool kTraceDefault = true;
#else
constexpr bool kTraceDefault = false;
#endif

std::mutex& fault_mu() {
  static std::mutex m;
  return m;
}

std::set<std::string>& fault_set() {
  static std::set<std::string> s = [] {
    std::set<std::string> r;
    if (const char* e = std::getenv("NTXENT_FAULT")) {
      std::stringstream ss(e);
      std::string tok;
      while (std::getline(ss, tok, ',')) if (!tok.empty()) r.insert(tok);
    }
    return r;
  }();
  return s;
}

// rocprofiler-sdk roctx entry points, resolved at run time: torch already loads the legacy
// libroctx64 which exports the same symbol names, so a link-time binding could land on it.
struct Roctx {
  using PushFn = int (*)(const char*);
  using PopFn = int (*)();
  using MarkFn = void (*)(const char*);
  PushFn push = nullptr;
  PopFn pop = nullptr;
  MarkFn mark = nullptr;
  Roctx() {
    void* lib = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!lib) lib = dlopen("/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!lib) return;
    push = reinterpret_cast<PushFn>(dlsym(lib, "roctxRangePushA"));
    pop = reinterpret_cast<PopFn>(dlsym(lib, "roctxRangePop"));
    mark = reinterpret_cast<MarkFn>(dlsym(lib, "roctxMarkA"));
  }
};

const Roctx& roctx() {
  static const Roctx r;
  return r;
}

}  // namespace

bool trace_enabled() {
  static const bool on = env_flag("NTXENT_ROCTX", kTraceDefault) && roctx().push && roctx().pop;
  return on;
}

void trace_push(const char* name) { roctx().push(name); }
void trace_pop() { roctx().pop(); }
void trace_mark(const char* name) {
  if (trace_enabled() && roctx().mark) roctx().mark(name);
}

bool fault_armed(const char* site) {
  std::lock_guard<std::mutex> g(fault_mu());
  const auto& s = fault_set();
  return !s.empty() && s.count(site) > 0;
}

void fault_point(const char* site) {
  if (fault_armed(site)) throw InjectedFault(site);
}

void set_fault_sites(const std::string& csv) {
  std::lock_guard<std::mutex> g(fault_mu());
  auto& s = fault_set();
  s.clear();
  std::stringstream ss(csv);
  std::string tok;
  while (std::getline(ss, tok, ',')) if (!tok.empty()) s.insert(tok);
}

}  // namespace ntxent
