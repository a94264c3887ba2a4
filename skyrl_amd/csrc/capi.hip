// C-ABI plumbing: thread-local error text, ABI version, launch checks.
#include "common.h"

namespace skyrl {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        return fail(SKYRL_ERR_LAUNCH, std::string(what) + ": " + hipGetErrorString(e));
    }
    return SKYRL_OK;
}

}  // namespace skyrl

extern "C" const char* skyrl_last_error(void) { return skyrl::g_last_error.c_str(); }

extern "C" int skyrl_abi_version(void) { return 12; }
