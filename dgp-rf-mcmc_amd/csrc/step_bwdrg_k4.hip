// step_bwdrg_k4.hip — k_step_bwd_rg instances with KS = 4 A-tile k-steps (layer input width d <= 16).
#define DGPRF_KS 4
#include "step_bwdrg_impl.h"
