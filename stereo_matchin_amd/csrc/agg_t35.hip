// aggregation passes for T = 35 taps (see asw_aggregate_impl.h)
#include "asw_aggregate_impl.h"
ASW_INSTANTIATE_PASS(35)
