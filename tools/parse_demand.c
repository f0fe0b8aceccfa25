/*
 * How much of k_match's work the parse consumes (VERDICT r2 "next" 1).
 * Builds the oracle restatement with its JDO_STATS hooks and deflates
 * 64 KiB blocks of a corpus at a level; counts the getmatch2 calls (the
 * records the lazy parse reads: fresh = threshold 2, lazy = threshold
 * prevlen - 1 at half budget), the chain hops of those calls, and the hops a
 * threshold-2 full-budget walk takes at every position the parse skips.
 *   gcc -O2 -o /tmp/pd tools/parse_demand.c jdeflate_amd/csrc/corpus.c -lpthread
 *   /tmp/pd text 6 64     (corpus, level, MiB)
 */
#define JDO_STATS 1
#include "../oracle/jdoracle.c"

void jdc_text(uint8_t* out, size_t n, uint64_t seed, int threads);
void jdc_mixed(uint8_t* out, size_t n, size_t blocksize, uint64_t seed, int threads);

static uint64_t n_fresh, n_lazy, h_fresh, h_lazy, n_skip, h_skip, n_steps, n_obs;
static uint64_t hist[8];
void jdo_stat_step(int hasmatch) { (void) hasmatch; n_steps++; }
void jdo_stat_obs(int a, int b, size_t c) { (void) a; (void) b; (void) c; n_obs++; }
void jdo_stat_call(int lazy, uint32_t hops, uint32_t len)
{
    (void) len;
    if (lazy) { n_lazy++; h_lazy += hops; } else { n_fresh++; h_fresh += hops; }
}
void jdo_stat_skip(uint32_t hops)
{
    n_skip++;
    h_skip += hops;
    hist[hops == 0 ? 0 : hops < 4 ? 1 : hops < 16 ? 2 : hops < 64 ? 3 : hops < 256 ? 4 : 5]++;
}

int main(int argc, char** argv)
{
    const char* kind = argc > 1 ? argv[1] : "text";
    const int level = argc > 2 ? atoi(argv[2]) : 6;
    const size_t n = (size_t) (argc > 3 ? atoi(argv[3]) : 64) << 20;
    uint8_t* src = malloc(n);
    uint8_t* dst = malloc(70000);
    if (!strcmp(kind, "text")) jdc_text(src, n, 1000, 8);
    else jdc_mixed(src, n, 65536, 1000, 8);
    for (size_t o = 0; o < n; o += 65536) jdo_deflate(src + o, 65536, level, 0, JDO_FLUSH, dst, 70000);
    const uint64_t calls = n_fresh + n_lazy;
    printf("%s L%d %zu MiB: positions %zu\n", kind, level, n >> 20, n);
    printf("  getmatch2 calls %llu (%.1f%% of positions): fresh %llu, lazy %llu\n",
           (unsigned long long) calls, 100.0 * calls / n, (unsigned long long) n_fresh,
           (unsigned long long) n_lazy);
    printf("  positions visited (fresh calls) %.1f%%; skipped %llu (%.1f%%)\n",
           100.0 * n_fresh / n, (unsigned long long) n_skip, 100.0 * n_skip / n);
    printf("  hops per call: fresh %.2f, lazy %.2f; hops per skipped position (full walk) %.2f\n",
           (double) h_fresh / (n_fresh ? n_fresh : 1), (double) h_lazy / (n_lazy ? n_lazy : 1),
           (double) h_skip / (n_skip ? n_skip : 1));
    printf("  share of all-positions hops at positions the parse reads: %.1f%%\n",
           100.0 * (h_fresh + h_lazy) / (double) (h_fresh + h_lazy + h_skip));
    printf("  skipped-position hop histogram: 0 %llu, 1-3 %llu, 4-15 %llu, 16-63 %llu, 64-255 %llu, 256+ %llu\n",
           (unsigned long long) hist[0], (unsigned long long) hist[1], (unsigned long long) hist[2],
           (unsigned long long) hist[3], (unsigned long long) hist[4], (unsigned long long) hist[5]);
    return 0;
}
