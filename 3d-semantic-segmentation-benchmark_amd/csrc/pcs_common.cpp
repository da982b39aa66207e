// Error plumbing of the C ABI: a thread-local last-error string.
#include "pcs_common.hpp"

#include <stdarg.h>

namespace {
thread_local char g_err[512] = "";
}

namespace pcs {

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int launch_status(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: launch failed: %s", what, hipGetErrorString(e));
        return (int)e;
    }
    return 0;
}

}  // namespace pcs

PCS_API const char* pcs_last_error(void) { return g_err; }

PCS_API int pcs_abi_version(void) { return 4; }

PCS_API int pcs_operand_size(void) { return (int)sizeof(pcs_operand); }

PCS_API int pcs_mlp_layer_size(void) { return (int)sizeof(pcs_mlp_layer); }
