// step_bwdrg_k2.hip — k_step_bwd_rg instances with KS = 2 A-tile k-steps (layer input width d <= 8).
#define DGPRF_KS 2
#include "step_bwdrg_impl.h"
