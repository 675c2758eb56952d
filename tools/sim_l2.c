// Set-associative LRU model of ONE XCD's L2 over the aggregation kernel's
// gather stream (CSR column array from tools/sim_l2_gen.py).  The XCD works on
// one feature tile; `share` XCDs split the tasks of that tile in blocks of
// `block_slots` slots (the kernel's b % 8 placement).  Capacity is in row
// tiles (4 MiB / tile bytes).  Calibrated against PMC: 64-feature tiles on
// two XCDs -> 32.6% (measured 33.2%), 128-feature tiles -> 22.5% (23.8%),
// 32-feature tiles on one XCD -> 44.6% (43.5%, profiles/r02_pmc_ab_slot_pairs.json).
//   gcc -O2 -o /tmp/sim_l2 tools/sim_l2.c
//   /tmp/sim_l2 <capacity_rows> <share> <block_slots> [bypass_outdeg] [ways]   (reads $SIM_COL or /tmp/sim/col.bin)
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
static int32_t *col; static int64_t E; static int N = 1<<21;
int main(int argc, char** argv){
  int cap = atoi(argv[1]); int share = atoi(argv[2]); int64_t blk = atoll(argv[3]);
  int bypass = argc > 4 ? atoi(argv[4]) : -1; int ways = argc > 5 ? atoi(argv[5]) : 16;
  const char* path = getenv("SIM_COL") ? getenv("SIM_COL") : "/tmp/sim/col.bin";
  FILE* f = fopen(path, "rb");
  if (!f) { fprintf(stderr, "cannot open %s\n", path); return 1; } fseek(f,0,SEEK_END); E = ftell(f)/4; fseek(f,0,SEEK_SET);
  col = malloc(E*4); if (fread(col,4,E,f) != (size_t)E) return 1; fclose(f);
  int* deg = calloc(N,4); for (int64_t i=0;i<E;i++) deg[col[i]]++;
  // set-associative LRU: sets = cap/ways, per set arrays of tags + stamps
  int sets = cap / ways;
  int32_t* tag = malloc((size_t)sets*ways*4); int64_t* st = malloc((size_t)sets*ways*8);
  memset(tag, 0xff, (size_t)sets*ways*4); memset(st, 0, (size_t)sets*ways*8);
  int64_t hits=0, acc=0, t=0;
  // XCD 0 of `share` XCDs working on the tile: it takes blocks k*share of size blk
  for (int64_t b0 = 0; b0 < E; b0 += blk*share) {
    int64_t e1 = b0 + blk < E ? b0 + blk : E;
    for (int64_t e = b0; e < e1; e++) {
      int r = col[e]; acc++; t++;
      uint32_t h = (uint32_t)r * 2654435761u; int s = (h >> 7) % sets;
      int32_t* tg = tag + (size_t)s*ways; int64_t* ss = st + (size_t)s*ways;
      int hit=-1, lru=0;
      for (int w=0; w<ways; w++){ if (tg[w]==r){hit=w;break;} if (ss[w]<ss[lru]) lru=w; }
      if (hit>=0){ hits++; ss[hit]=t; }
      else if (deg[r] > bypass){ tg[lru]=r; ss[lru]=t; }
    }
  }
  printf("cap=%d share=%d blk=%lld bypass=%d ways=%d: hit %.3f (acc %lld)\n", cap, share, (long long)blk, bypass, ways, (double)hits/acc, (long long)acc);
  return 0;
}
