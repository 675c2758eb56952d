// Cache model of the config-2 aggregation for destination-row processing
// orders: all 8 XCD L2s plus the shared 256 MiB Infinity
// Cache (MALL), over the kernel's gather stream.
//
//   * feature tiles: 4 tiles of 64 features (256 B per gathered row tile); tile t
//     runs on XCDs t and t+4 (the kernel's XCD-affine map), which take its task
//     blocks alternately (blocks of `blk` slots, the b % 8 placement);
//   * a destination-row ORDER (int32 permutation, one file) sets the sequence in
//     which rows are processed; each row's slots keep their CSR order (outputs
//     are still written to the original row ids, so this is a schedule only);
//   * L2: 4 MiB per XCD = 16384 row tiles, 16-way set-associative LRU, keyed by
//     the source row (an XCD holds one tile);
//   * IC: 256 MiB shared = 1M row tiles, 16-way LRU, keyed by (row, tile); it
//     sees every L2 miss of every XCD;
//   * the 8 XCD streams advance round-robin one gather at a time (equal progress).
// mode "split": the XCD pair of a tile splits the SOURCES (even / odd column)
// instead of the task blocks: each XCD walks every row, gathering only its half
// (the cross-XCD source split of DESIGN 3.9; costs a partial-row combine).
//   gcc -O2 -o /tmp/sim_orders tools/sim_orders.c
//   /tmp/sim_orders <order.bin | -> [blk] [split]     (reads /tmp/sim/col.bin, rowptr.bin)
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  int sets, ways;
  int64_t* tag;
  int64_t* st;
} Cache;

static void cache_init(Cache* c, int64_t entries, int ways) {
  c->ways = ways;
  c->sets = (int)(entries / ways);
  c->tag = malloc(sizeof(int64_t) * c->sets * ways);
  c->st = calloc((size_t)c->sets * ways, sizeof(int64_t));
  memset(c->tag, 0xff, sizeof(int64_t) * c->sets * ways);
}

// returns 1 on hit; inserts on miss (LRU)
static int cache_access(Cache* c, int64_t key, int64_t t) {
  uint64_t h = (uint64_t)key * 0x9E3779B97F4A7C15ull;
  int s = (int)((h >> 29) % (uint64_t)c->sets);
  int64_t* tg = c->tag + (int64_t)s * c->ways;
  int64_t* ss = c->st + (int64_t)s * c->ways;
  int lru = 0;
  for (int w = 0; w < c->ways; w++) {
    if (tg[w] == key) {
      ss[w] = t;
      return 1;
    }
    if (ss[w] < ss[lru]) lru = w;
  }
  tg[lru] = key;
  ss[lru] = t;
  return 0;
}

static int32_t* load(const char* p, int64_t* n) {
  FILE* f = fopen(p, "rb");
  if (!f) {
    fprintf(stderr, "cannot open %s\n", p);
    exit(1);
  }
  fseek(f, 0, SEEK_END);
  *n = ftell(f) / 4;
  fseek(f, 0, SEEK_SET);
  int32_t* a = malloc(*n * 4);
  if (fread(a, 4, *n, f) != (size_t)*n) exit(1);
  fclose(f);
  return a;
}

int main(int argc, char** argv) {
  int64_t E, N1, NO = 0;
  int32_t* col = load("/tmp/sim/col.bin", &E);
  int32_t* rowptr = load("/tmp/sim/rowptr.bin", &N1);
  const int64_t N = N1 - 1;
  int32_t* order = NULL;
  if (argc > 1 && strcmp(argv[1], "-") != 0) order = load(argv[1], &NO);
  const int64_t blk = argc > 2 ? atoll(argv[2]) : 4096;
  const int split = argc > 3 && strcmp(argv[3], "split") == 0;
  // the processed slot sequence: rows in order, each row's slots in CSR order
  int32_t* seq = malloc(E * 4);
  int64_t k = 0;
  for (int64_t i = 0; i < N; i++) {
    int64_t r = order ? order[i] : i;
    for (int64_t e = rowptr[r]; e < rowptr[r + 1]; e++) seq[k++] = col[e];
  }
  Cache l2[8], ic;
  for (int x = 0; x < 8; x++) cache_init(&l2[x], 16384, 16);
  cache_init(&ic, 1 << 20, 16);
  // per XCD cursor over its share of the tile's stream
  int64_t pos[8], l2h = 0, ich = 0, acc = 0, t = 0;
  for (int x = 0; x < 8; x++) pos[x] = split ? 0 : (x / 4) * blk;
  int live = 8;
  while (live > 0) {
    live = 0;
    for (int x = 0; x < 8; x++) {
      int64_t p = pos[x];
      if (split) {  // every slot of the stream, keep this XCD's parity of sources
        while (p < E && (seq[p] & 1) != (x / 4)) p++;
      }
      if (p >= E) {
        pos[x] = p;
        continue;
      }
      live++;
      const int64_t r = seq[p];
      const int tile = x % 4;
      acc++;
      t++;
      if (cache_access(&l2[x], r, t)) {
        l2h++;
      } else if (cache_access(&ic, r * 4 + tile, t)) {
        ich++;
      }
      p++;
      if (!split && (p % blk) == 0) p += blk;  // skip the other XCD's block
      pos[x] = p;
    }
  }
  const double h = (double)l2h / acc, ic_of_miss = (double)ich / (acc - l2h);
  printf("order=%s blk=%lld%s: gathers %lld  L2 hit %.4f  IC hit (of L2 misses) %.4f  HBM %.4f\n",
         argc > 1 ? argv[1] : "-", (long long)blk, split ? " src-split" : "", (long long)acc, h, ic_of_miss,
         (1 - h) * (1 - ic_of_miss));
  return 0;
}
