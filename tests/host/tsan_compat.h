// tsan_compat.h — TEST ONLY, force-included in the ThreadSanitizer build of queue_host.cpp.
// GCC 11's libtsan does not intercept pthread_cond_clockwait, which libstdc++ uses for
// std::condition_variable::wait_until/wait_for on steady_clock: TSan then misses the unlock/relock inside
// the wait and reports a false "double lock". Without the macro libstdc++ uses pthread_cond_timedwait,
// which TSan does intercept. The queue code itself is unchanged.
#include <bits/c++config.h>
#undef _GLIBCXX_USE_PTHREAD_COND_CLOCKWAIT
