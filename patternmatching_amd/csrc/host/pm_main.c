/*
 * pm_main.c -- the `pm` command line, a drop-in for the reference's `exe`
 * (Core/src/main.c:7-24): same -d/-s/-o/-v surface, same phases
 * (setup, parse arguments, build the matchers, measure, write the CSV).
 */
#include <stdio.h>
#include <stdlib.h>
#include "pm_host.h"
#include "pm_hip.h"

int main(int argc, char** argv) {
    PmConf conf;
    PmInstanceStats stats[PM_MPS_SIZE];
    char err[512];
    pm_mps_table_setup();
    if (pm_parse_args(argc, argv, &conf) != 0) return EXIT_FAILURE;
    if (pm_hip_device_count() <= conf.device) {
        fprintf(stderr, "pm: no HIP device %d (found %d); this build has no CPU fallback\n", conf.device,
                pm_hip_device_count());
        return EXIT_FAILURE;
    }
    pm_hip_set_device(conf.device);
    printf("\nInitializing Multi-Pattern Search engine\n");
    PmDict* dict = pm_dict_load((const char* const*)conf.dict_files, conf.n_dict_files, err, sizeof(err));
    if (!dict) {
        fprintf(stderr, "%s\n", err);
        return EXIT_FAILURE;
    }
    if (conf.verbose)
        printf("%zu unique patterns (max length %zu) from %zu lines\n", dict->n, dict->max_len, dict->lines_total);
    printf("\nStart the Algorithms measuring\n");
    if (pm_measure_all(&conf, dict, stats) != 0) return EXIT_FAILURE;
    if (pm_write_stats(&conf, stats) != 0) return EXIT_FAILURE;
    printf("\nprogram done\n");
    pm_dict_free(dict);
    pm_conf_free(&conf);
    return 0;
}
