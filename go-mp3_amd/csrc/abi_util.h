// abi_util.h -- shared helpers of the C-ABI translation units.
#pragma once

namespace mp3g {
// Records `what` as this thread's mp3g_last_error() text and returns status.
int abi_fail(int status, const char* what);
// Whether the plan kernel of `mode` reads only coefficient lines below count1
// (fast v3, exact v4): the main-data kernel may then skip the zero tails
// (MP3G_HUFF_ROWS_COUNT1).
bool mode_reads_to_count1(unsigned mode);
}  // namespace mp3g
