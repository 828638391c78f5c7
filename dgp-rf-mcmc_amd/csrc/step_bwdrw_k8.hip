// step_bwdrw_k8.hip — k_step_bwd_rw instances with KS = 8 A-tile k-steps (layer input width d <= 32).
#define DGPRF_KS 8
#include "step_bwdrw_impl.h"
