// cimq_part_v7_88.hip -- the v7 backward for w8a8 layers (nbw = nba = 8).
#include "cimq_v7_launch.h"

namespace cimq {
template CIMQ_V7_SIG(8, 8);
}  // namespace cimq
