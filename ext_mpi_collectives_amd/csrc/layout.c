/*
 * layout.c -- turns owner chunks into device launch layouts (host C, no HIP calls):
 * alignment split of each bucket, tile numbering of the streaming kernel, and the
 * element-granular edge items. Shared by the engine and the one-chunk device ABI.
 */
#include <stdlib.h>

#include "gpu.h"

/* head / vector / tail split of one bucket whose pointers are at element 0 of the chunk:
   vectors need every pointer 16-byte aligned at the same element; if they disagree the whole
   bucket is element-granular (edge path). On return the pointers sit at element `head`, the
   first full vector, so the streaming kernel adds no offset. */
void emac_split_alignment(emac_bucket *b, int nsrc, long len, int tsize) {
  long head = 0;
  int i, ok = 1;
  unsigned long mis = (unsigned long)b->src[0] & 15ul;
  if (mis % (unsigned long)tsize == 0)
    head = (long)((16ul - mis) & 15ul) / tsize;
  else
    ok = 0;
  if (head > len) head = len;
  for (i = 0; ok && i < nsrc; i++)
    if (((unsigned long)((const char *)b->src[i] + head * tsize) & 15ul) != 0) ok = 0;
  for (i = 0; ok && i < b->ndst; i++)
    if (((unsigned long)((char *)b->dst[i] + head * tsize) & 15ul) != 0) ok = 0;
  b->count = len;
  if (!ok) {
    b->scalar = 1;
    b->head = b->tail = b->nvec = 0;
    return;
  }
  b->scalar = 0;
  b->head = head;
  b->nvec = (len - head) * tsize / 16;
  b->tail = len - head - b->nvec * (16 / tsize);
  for (i = 0; i < nsrc; i++) b->src[i] = (const char *)b->src[i] + head * tsize;
  for (i = 0; i < b->ndst; i++) b->dst[i] = (char *)b->dst[i] + head * tsize;
}

int emac_tree_kind(const emac_codes *c, int op) {
  static const int chains[] = EMAC_CHAINS;
  int rad[EMAC_MAX_LEVELS], l, t, g = 1, ch = 0;
  unsigned k;
  if (c->nlev <= 1) return 0;
  if (op != EMAC_SUM || c->nlev > 4) return 1;
  /* level-l group size = 1 + the first leaf that closes level l (plan.c build_codes) */
  for (l = 0; l < c->nlev; l++) {
    for (t = 0; t < c->nleaf && c->close[t] <= l; t++);
    if (t == c->nleaf || (t + 1) % g) return 1;
    rad[l] = (t + 1) / g;
    g = t + 1;
    if (rad[l] < 2 || rad[l] > 31) return 1;
    ch |= rad[l] << (5 * l);
  }
  if (g != c->nleaf) return 1;
  for (k = 0; k < sizeof(chains) / sizeof(chains[0]); k++)
    if (chains[k] == ch) return ch;
  return 1;
}

int emac_layout(emac_bucket *b, int nb, int op, int nsrc, int tree, int fan, emac_edge **edges_out, int *nedges,
                long *ntiles_out, long *tpb_out, int *all_full_out, int *unroll_out) {
  return emac_layout_as(b, nb, op, nsrc, tree, fan, 0, edges_out, nedges, ntiles_out, tpb_out, all_full_out, unroll_out);
}

int emac_layout_as(emac_bucket *b, int nb, int op, int nsrc, int tree, int fan, int forced, emac_edge **edges_out,
                   int *nedges, long *ntiles_out, long *tpb_out, int *all_full_out, int *unroll_out) {
  long total = 0, tv, tiles = 0, uniform = -1;
  int i, ne = 0, unroll, all_full = 1;
  emac_edge *edges;
  for (i = 0; i < nb; i++) total += b[i].nvec;
  unroll = forced > 0 ? forced : emac_gpu_pick_unroll(op, nsrc, tree, fan, total); /* U | ISSUE << 4 */
  tv = (long)EMAC_BLOCK * (unroll & 15);
  for (i = 0; i < nb; i++) {
    long t = (b[i].nvec + tv - 1) / tv;
    b[i].tile0 = tiles;
    tiles += t;
    uniform = (uniform == -1 || uniform == t) ? t : 0;
    if (b[i].nvec % tv) all_full = 0;
    if (b[i].scalar)
      ne += (int)((b[i].count + EMAC_EDGE_RANGE - 1) / EMAC_EDGE_RANGE);
    else if (b[i].head + b[i].tail > 0)
      ne++;
  }
  edges = (emac_edge *)malloc(sizeof(emac_edge) * (size_t)(ne + 1));
  if (!edges) return EMAC_ERR_MALLOC;
  ne = 0;
  for (i = 0; i < nb; i++) {
    if (b[i].scalar) {
      long s;
      for (s = 0; s < b[i].count; s += EMAC_EDGE_RANGE) {
        edges[ne].bucket = i;
        edges[ne].mode = 1;
        edges[ne].start = s;
        edges[ne].count = b[i].count - s < EMAC_EDGE_RANGE ? b[i].count - s : EMAC_EDGE_RANGE;
        ne++;
      }
    } else if (b[i].head + b[i].tail > 0) {
      edges[ne].bucket = i;
      edges[ne].mode = 0;
      edges[ne].start = 0;
      edges[ne].count = b[i].head + b[i].tail;
      ne++;
    }
  }
  *edges_out = edges;
  *nedges = ne;
  *ntiles_out = tiles;
  *tpb_out = uniform > 0 ? uniform : 0;
  {
    /* a leaf-major deferred-store schedule (fold_kernel.hpp kDeferShift: groups of kb tiles of one bucket) over
       buckets of unequal tile counts, at most EMAC_GROUP_MAP_MAX of them (the `-k` fractions: a few
       short chunks beside one long one): each bucket's tile0 becomes its first GROUP, ntiles the
       groups of the launch and tiles_per_bucket -1 -- the kernel finds a group's bucket in a table
       of these starts it keeps in LDS, instead of falling back to the per-tile loop */
    const int issue = unroll >> 4, kd = (issue >> 11) & 3;
    const long kb = kd ? 1L << kd : 1;
    if (kb > 1 && (issue & (1 << 13)) && *tpb_out == 0 && nb > 0 && nb <= EMAC_GROUP_MAP_MAX) { /* leaf-major (kLeafMajor) */
      long g = 0;
      for (i = 0; i < nb; i++) {
        b[i].tile0 = g;
        g += ((b[i].nvec + tv - 1) / tv + kb - 1) / kb;
      }
      *ntiles_out = g;
      *tpb_out = -1;
    }
  }
  *all_full_out = all_full;
  *unroll_out = unroll;
  return 0;
}
