// at2v_env.h — the library's environment hooks, gated (VERDICT r5 "What's weak" 8).
//
// The library reads test and A/B knobs from the environment (device aliasing, injected launch / communicator failures,
// forced fingerprint collisions, scratch sets, queue variants, staging sizes), but only in a process that opted in with
// AT2V_TEST_HOOKS=1: a production node whose environment happens to carry one of these names behaves exactly as if it
// did not. tests/conftest.py and the tools/ recipes set the gate; bench.py does not.
#pragma once
#include <cstdlib>
#include <cstring>

namespace at2v {

inline bool test_hooks_enabled() {
  const char* v = std::getenv("AT2V_TEST_HOOKS");
  return v && std::strcmp(v, "1") == 0;
}

// getenv(name) when the hooks are enabled, else nullptr (read at context / queue creation, never per launch)
inline const char* test_env(const char* name) { return test_hooks_enabled() ? std::getenv(name) : nullptr; }

inline long test_env_long(const char* name, long dflt) {
  const char* v = test_env(name);
  return v ? std::strtol(v, nullptr, 10) : dflt;
}

}  // namespace at2v
