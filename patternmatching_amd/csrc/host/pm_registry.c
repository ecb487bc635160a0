/*
 * pm_registry.c -- the plugin table (Core/src/mps.c:29, :120-124).
 * Each algorithm's register function fills its slot, as mps_ac_register
 * does (Core/src/mpac.c:358-367).
 */
#include "pm_mps.h"
#include "pm_hip.h"

PmMpsElem pm_mps_table[PM_MPS_SIZE];

void pm_mps_table_setup(void) {
    pm_mps_hip_rt_register(&pm_mps_table[PM_MPS_HIP_RT]);
    pm_mps_hip_ac_register(&pm_mps_table[PM_MPS_HIP_AC]);
    pm_mps_hip_auto_register(&pm_mps_table[PM_MPS_HIP_AUTO]);
}
