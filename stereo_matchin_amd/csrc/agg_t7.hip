// aggregation passes for T = 7 taps (see asw_aggregate_impl.h)
#include "asw_aggregate_impl.h"
ASW_INSTANTIATE_PASS(7)
