// step_bwd_k4.hip — k_step_bwd instances with KS = 4 A-tile k-steps (layer input width d <= 16).
#define DGPRF_KS 4
#include "step_bwd_impl.h"
