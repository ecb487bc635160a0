/*
 * ref_loop.c -- TEST INFRASTRUCTURE ONLY.
 *
 * The reference's own program (Core/src/main.c) with the HIP plugin
 * registered: mps_table_setup() (mps.c:120-124), then the stub of
 * oracle/mphip.c puts a libpm.so kind into an existing table slot, then
 * the reference's unmodified parse_arguments (parser.c:103), init_mps
 * (mps.c:109-113), measure_instances_stats (measure.c:324-332: reset per
 * stream file, read_char per byte at :292-294, the reliable AC instance and
 * measure_success_rate at :300-303) and write_stats_to_file (measure.c:339).
 * Only this file and mphip.c are ours; every other object is the
 * reference's, compiled where it lies by oracle/Makefile.
 *
 *   PM_REF_BG=rt|ac|auto    kind in the MPS_BG slot   (default rt)
 *   PM_REF_LMAC=rt|ac|auto  kind in the MPS_LMAC slot (default: the reference's LMAC)
 *   ref_loop -d DICT -s STREAM -o OUT.csv [-v]
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "conf.h"
#include "measure.h"
#include "mps.h"
#include "parser.h"
#include "util.h"

int mps_hip_register_into(int slot, const char* kind);

int main(int argc, char** argv) {
    program_name = argv[0];
    Conf* conf = (Conf*)calloc(1, sizeof(Conf));
    if (conf == NULL) {
        perror("failed to allocate memory");
        FatalExit();
    }
    mps_table_setup();
    const char* bg = getenv("PM_REF_BG");
    const char* lmac = getenv("PM_REF_LMAC");
    if (mps_hip_register_into(MPS_BG, bg ? bg : "rt") != 0 || (lmac && mps_hip_register_into(MPS_LMAC, lmac) != 0)) {
        fprintf(stderr, "ref_loop: unknown HIP kind\n");
        return 2;
    }
    parse_arguments(argc, argv, conf);
    init_mps(conf);
    measure_instances_stats(conf);
    write_stats_to_file(conf);
    return 0;
}
