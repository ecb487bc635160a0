/*
 * mphip.c -- the registration stub of INTEGRATION.md §2, as a compiled file.
 * TEST INFRASTRUCTURE here: oracle/ref_loop.c links it with the reference's
 * own objects and libpm.so.  A reference maintainer would add it as
 * Core/src/mphip.c (pattern: mps_ac_register, Core/src/mpac.c:358-367).
 *
 * With the enum edit of INTEGRATION.md §2 (MPS_HIP_RT / MPS_HIP_AC /
 * MPS_HIP_AUTO before MPS_SIZE, mps.h:20-25) mps_hip_register() fills those
 * three slots.  Against the unmodified reference -- how the tests run it --
 * mps_hip_register_into() puts one HIP kind into an existing slot (the MPBG
 * slot: MPBG is randomized and O(patterns) per byte).
 * MpsElem has no read_block member unless the maintainer adds it
 * (MPS_ELEM_HAS_READ_BLOCK); the reference's loop then calls read_char per
 * byte (measure.c:292-294), which libpm.so serves with its host step.
 */
#include <string.h>

#include "mps.h"
#include "pm_hip.h" /* -I<this repo>/include */

static void reg(MpsElem* e, char* name, void* (*create)(void)) {
    e->name = name;
    e->create = create;
    e->add_pattern = (void (*)(void*, char*, size_t, pattern_id_t))pm_hip_add_pattern;
    e->compile = pm_hip_compile;
    e->read_char = (pattern_id_t(*)(void*, char))pm_hip_read_char;
    e->total_mem = pm_hip_total_mem;
    e->reset = pm_hip_reset;
    e->free = pm_hip_free;
#ifdef MPS_ELEM_HAS_READ_BLOCK
    e->read_block = (void (*)(void*, const char*, size_t, pattern_id_t*))pm_hip_read_block;
#endif
}

#ifdef MPS_HIP_RT
void mps_hip_register(void) {
    reg(&mps_table[MPS_HIP_RT], "HIP Reverse-Trie", pm_hip_rt_create);
    reg(&mps_table[MPS_HIP_AC], "HIP Aho-Corasick DFA", pm_hip_ac_create);
    reg(&mps_table[MPS_HIP_AUTO], "HIP Auto (RT / AC per launch)", pm_hip_auto_create);
}
#endif

#ifdef PM_READ_BLOCK_HOOK
/* the batch entry per slot that oracle/batch_measure.py's edit of the
 * reference's loop calls (NULL: read_char per byte) */
void (*mps_read_block[MPS_SIZE])(void*, const char*, size_t, pattern_id_t*);
#endif

/* kind: "rt", "ac" or "auto"; returns 0, or -1 for an unknown kind */
int mps_hip_register_into(int slot, const char* kind) {
    if (!strcmp(kind, "rt")) reg(&mps_table[slot], "HIP Reverse-Trie", pm_hip_rt_create);
    else if (!strcmp(kind, "ac")) reg(&mps_table[slot], "HIP Aho-Corasick DFA", pm_hip_ac_create);
    else if (!strcmp(kind, "auto")) reg(&mps_table[slot], "HIP Auto (RT / AC per launch)", pm_hip_auto_create);
    else return -1;
#ifdef PM_READ_BLOCK_HOOK
    mps_read_block[slot] = (void (*)(void*, const char*, size_t, pattern_id_t*))pm_hip_read_block;
#endif
    return 0;
}
