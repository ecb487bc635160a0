/*
 * abi_check.c -- TEST INFRASTRUCTURE ONLY (compiled, never linked or run).
 *
 * Compile-time proof that the drop-in boundary's table slot is layout-
 * compatible with the reference's: include/pm_mps.h's PmMpsElem begins with
 * exactly the eight members of MpsElem (Core/src/mps.h:71-80), in order and
 * at the same offsets, and pm_pattern_id_t has the size of pattern_id_t
 * (PatternsTree.h:104).  tests/test_integration.py compiles it with
 *   gcc -fsyntax-only -I/root/reference/Core/src -Iinclude oracle/abi_check.c
 * against the reference's own headers, where they lie.
 */
#include <stddef.h>

#include "mps.h"     /* the reference's (Core/src/mps.h) */
#include "pm_mps.h"  /* ours (include/pm_mps.h) */

_Static_assert(sizeof(pattern_id_t) == sizeof(pm_pattern_id_t), "pattern id size");
_Static_assert(_Alignof(pattern_id_t) == _Alignof(pm_pattern_id_t), "pattern id alignment");
_Static_assert(offsetof(PmMpsElem, read_block) == sizeof(MpsElem), "read_block follows the MpsElem prefix");
_Static_assert(_Alignof(PmMpsElem) == _Alignof(MpsElem), "slot alignment");

#define SAME_MEMBER(m)                                                                            \
    _Static_assert(offsetof(MpsElem, m) == offsetof(PmMpsElem, m), "offset of " #m);             \
    _Static_assert(sizeof(((MpsElem*)0)->m) == sizeof(((PmMpsElem*)0)->m), "size of " #m)

SAME_MEMBER(name);
SAME_MEMBER(create);
SAME_MEMBER(add_pattern);
SAME_MEMBER(compile);
SAME_MEMBER(read_char);
SAME_MEMBER(total_mem);
SAME_MEMBER(reset);
SAME_MEMBER(free);

/* the members' function types, with pattern_id_t in the reference's
 * signatures standing for pm_pattern_id_t (both opaque pointers) */
static void check_types(MpsElem* e, PmMpsElem* p) {
    char* (*name) = &e->name;
    void* (**create)(void) = &p->create;
    void (**compile)(void*) = &p->compile;
    size_t (**total_mem)(void*) = &p->total_mem;
    void (**reset)(void*) = &p->reset;
    void (**free_)(void*) = &p->free;
    void (**add)(void*, char*, size_t, pattern_id_t) = &e->add_pattern;
    pattern_id_t (**rc)(void*, char) = &e->read_char;
    e->create = *create;
    e->compile = *compile;
    e->total_mem = *total_mem;
    e->reset = *reset;
    e->free = *free_;
    (void)name;
    (void)add;
    (void)rc;
}

/* the MpsInstance pair too (mps.h:89-92) */
_Static_assert(sizeof(MpsInstance) == sizeof(PmMpsInstance), "instance size");
_Static_assert(offsetof(MpsInstance, obj) == offsetof(PmMpsInstance, obj), "instance obj");
_Static_assert(offsetof(MpsInstance, algo) == offsetof(PmMpsInstance, algo), "instance algo");

void pm_abi_check_unused(void) { check_types(0, 0); }
