// step_bwdrw_k4.hip — k_step_bwd_rw instances with KS = 4 A-tile k-steps (layer input width d <= 16).
#define DGPRF_KS 4
#include "step_bwdrw_impl.h"
