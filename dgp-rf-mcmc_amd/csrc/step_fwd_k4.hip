// step_fwd_k4.hip — k_step_fwd instances with KS = 4 A-tile k-steps (layer input width d <= 16).
#define DGPRF_KS 4
#include "step_fwd_impl.h"
