/* asan_node_programs.c -- host sanitizer pass over the inter-node planner (plan.c): every
   program of 22 EXT_MPI_NUM_PORTS lists x 6 copy-ins x 7 counts x every node and rank, built with
   gcc -fsanitize=address,undefined (no GPU, no preload):
     gcc -O1 -g -fsanitize=address,undefined -std=gnu11 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include \
       -Iinclude -Iext_mpi_collectives_amd/csrc ext_mpi_collectives_amd/csrc/plan.c tools/asan_node_programs.c
   Round 2: 12376 programs, no report, no leak. Round 3 adds the peer-mapped join's shares
   (emac_node_shares) of every node rank under every list it takes, each checked to tile the
   rank's chunk exactly once. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "plan.h"
int main(void) {
  static const int lists[][10] = {{-1, 1, 0}, {-1, -1, 1, 1, 0}, {-2, 2, 0}, {-3, 3, 0}, {-1, -2, 2, 1, 0},
                                  {-2, -1, 1, 2, 0}, {-3, -1, 1, 3, 0}, {-2, -2, 2, 2, 0}, {-1, -1, -1, 1, 1, 1, 0},
                                  {-4, 4, 0}, {3, 0}, {-1, 1, 1, 0}, {1, 1, 0}, {2, 0}, {-1, 2, 1, 0}, {-1, 3, 1, 0},
                                  {2, 1, 0}, {1, 0}, {-1, -1, 3, 0}, {-1, -1, -1, 3, 1, 0}, {-15, 15, 0}, {-1, -1, -1, -1, 1, 1, 1, 1, 0}};
  static const int nodes_of[] = {2, 4, 3, 4, 6, 6, 8, 9, 8, 5, 4, 4, 4, 3, 6, 8, 6, 2, 4, 8, 16, 16};
  static const char *copyins[] = {"6;1 -1 1", "6;1 -2 2", "6;1 -4 4", "6;3 -2 2", "6;-5 -2 2", "7;1 -2 2"};
  static const int Rs[] = {1, 2, 4, 2, 2, 2};
  long counts[] = {0, 1, 5, 7, 1031, 4099, 65543};
  int li, ci, k, node, me, n = 0, nsh_total = 0;
  for (li = 0; li < (int)(sizeof(nodes_of) / sizeof(int)); li++) {
    emac_node_sched ns;
    int rc = emac_node_sched_build(&ns, nodes_of[li], lists[li]);
    if (rc) { printf("list %d rejected %d\n", li, rc); continue; }
    for (ci = 0; ci < 6; ci++)
      for (k = 0; k < 7; k++) {
        emac_copyin cfg;
        emac_plan p;
        if (Rs[ci] == 1)
          emac_default_copyin(1, &cfg);
        else if (emac_parse_copyin(copyins[ci], &cfg)) { printf("parse fail %s\n", copyins[ci]); return 1; }
        cfg.sockets = 1;
        if (emac_plan_build(&p, Rs[ci], counts[k], EMAC_FLOAT, EMAC_SUM, &cfg)) continue;
        for (node = 0; node < nodes_of[li]; node++)
          for (me = 0; me < Rs[ci]; me++) {
            emac_p2p *ops; emac_fold *folds; int no, nf; long st;
            if (emac_comm_program_nodes(&p, &ns, node, me, 4, &ops, &no, &folds, &nf, &st)) { printf("prog fail\n"); return 1; }
            free(ops); free(folds); n++;
          }
        for (me = 0; me < Rs[ci] && emac_node_single(&ns); me++) {
          emac_share *sh; int nsh, i, pc; long covered = 0, want = 0;
          if (emac_node_shares(&p, &ns, me, &sh, &nsh)) { printf("shares fail\n"); return 1; }
          for (pc = 0; pc < p.npieces; pc++) want += p.chunk_len[(size_t)pc * Rs[ci] + p.rank_pos[me]];
          for (i = 0; i < nsh; i++) covered += sh[i].len;
          if (covered != want) { printf("shares cover %ld of %ld (list %d)\n", covered, want, li); return 1; }
          nsh_total += nsh;
          free(sh);
        }
        emac_plan_free(&p);
      }
  }
  printf("programs %d, shares %d\n", n, nsh_total);
  return 0;
}
