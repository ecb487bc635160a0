/*
 * pm_mps.h -- the multi-pattern-search plugin ABI, restated for the MI355X
 * build.  This is the drop-in boundary.
 *
 * Reference interface it mirrors:
 *   MpsElem            /root/reference/Core/src/mps.h:71-80
 *   MpsInstance        /root/reference/Core/src/mps.h:89-92
 *   mps_table[]        /root/reference/Core/src/mps.h:94, mps.c:29
 *   pattern_id_t       /root/reference/Core/src/PatternsTree.h:104 (a pointer)
 *   null_pattern_id    /root/reference/Core/src/PatternsTree.h:106 (NULL)
 *   read_char contract /root/reference/Core/src/mps.h:41-42,
 *                      /root/reference/Core/src/README.md:99-105
 *
 * Layout: the first eight members are exactly MpsElem's, in MpsElem's order,
 * so a PmMpsElem* can be used where the reference expects an MpsElem*.
 * `read_block` is the one extension (NULL for per-byte CPU plugins): it must
 * be identical to n successive read_char calls, with the matcher state
 * carried across calls and cleared only by reset.
 */
#ifndef PM_MPS_H
#define PM_MPS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Opaque, pointer-sized and compared with '==' exactly like the reference's
 * PatternsTreeNode* (PatternsTree.h:104).  Plugins return the id they were
 * given in add_pattern verbatim. */
typedef struct PmPattern* pm_pattern_id_t;
#define PM_NULL_PATTERN_ID ((pm_pattern_id_t)0)

typedef struct {
    char* name;
    void* (*create)(void);
    void (*add_pattern)(void*, char*, size_t, pm_pattern_id_t);
    void (*compile)(void*);
    pm_pattern_id_t (*read_char)(void*, char);
    size_t (*total_mem)(void*);
    void (*reset)(void*);
    void (*free)(void*);
    /* --- extension (after the MpsElem prefix) --- */
    void (*read_block)(void*, const char* buf, size_t n, pm_pattern_id_t* out);
} PmMpsElem;

typedef struct {
    void* obj;
    int algo;
} PmMpsInstance;

/* Algorithms of this build (mps.h:20-25 pattern: append before PM_MPS_SIZE).
 * All are GPU matchers with the exact read_char contract:
 *   PM_MPS_HIP_RT    reverse-suffix-trie walk, one lane per stream position
 *   PM_MPS_HIP_AC    Aho-Corasick dense DFA, one lane per stream segment
 *   PM_MPS_HIP_AUTO  both, the kernel picked per block by the RT kernel's
 *                    measured spill rate (dense deep matches -> AC) */
enum {
    PM_MPS_HIP_RT = 0,
    PM_MPS_HIP_AC,
    PM_MPS_HIP_AUTO,
    PM_MPS_SIZE
};

extern PmMpsElem pm_mps_table[PM_MPS_SIZE];

/* mps.c:120-124 equivalent: fill pm_mps_table. */
void pm_mps_table_setup(void);

#ifdef __cplusplus
}
#endif
#endif /* PM_MPS_H */
