// abi_util.h -- shared helpers of the C-ABI translation units.
#pragma once

namespace mp3g {
// Records `what` as this thread's mp3g_last_error() text and returns status.
int abi_fail(int status, const char* what);
}  // namespace mp3g
