// svo_hip.h — error plumbing shared by the HIP translation units (svo_cast.hip, svo_build.hip)
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "svo_internal.h"

#define SVO_FAIL(code, msg)     \
    do {                        \
        svo::set_error(msg);    \
        return (code);          \
    } while (0)

#define HIP_TRY(expr, code)                                                                    \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess) {                                                                \
            svo::set_error(std::string(#expr " failed: ") + hipGetErrorString(e_));            \
            return (code);                                                                     \
        }                                                                                      \
    } while (0)
