// Shared error state of the learner-side C ABI (flock_learn_last_error), used by every learner source file.
#pragma once

namespace flock_learn_internal {
extern thread_local char g_err[256];
int fail(int code, const char* msg);  // records msg, returns code
int launched();                       // 0, or -4 with the HIP error string of the last launch
}  // namespace flock_learn_internal
