// Force-included into the ThreadSanitizer build only (tools/tsan_build.sh). gcc 11's TSan runtime does not
// intercept pthread_cond_clockwait, which libstdc++ uses for condition_variable waits on steady_clock. TSan then
// misses the mutex release and re-acquire inside the wait, and reports double locks and races on data that the
// mutex guards. Undefining the configure macro after <bits/c++config.h> makes <condition_variable> use
// pthread_cond_timedwait, which TSan intercepts. Product builds do not include this file.
#pragma once
#include <bits/c++config.h>
#undef _GLIBCXX_USE_PTHREAD_COND_CLOCKWAIT
