/* kmatch_demand.c -- CPU model of a capped match pass with exact fixes on
 * demand (dev tool, not product).  Per 64 KiB block: every position's
 * getmatch2 walk (deflator.c:2650-2674, threshold 2) at full budget and cut
 * at C hops; then the lazy parse (compress2 :2826-2906, simplified: no
 * 3-chain candidate, no block split) over records that are exact only where
 * the capped walk ended on its own or a fix was made, repeated: every
 * position the parse read (token starts and the position after each match)
 * whose record was cut is fixed (full walk), until a parse reads no cut
 * record.  Prints the hops of the capped pass, the hops of the fixes, the
 * parse passes needed and the blocks needing each.
 *   gcc -O2 -o /tmp/kmd tools/kmatch_demand.c && /tmp/kmd file level cap
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint32_t head_be(const uint8_t* b, uint32_t p, uint32_t len)
{
    uint32_t v = 0;
    for (int k = 0; k < 4; k++) if (p + k < len) v |= (uint32_t) b[p + k] << (8 * k);
    return __builtin_bswap32(v);
}
static int ilog2(uint32_t x) { return 31 - __builtin_clz(x); }

static double S[16];
static uint64_t passes_hist[64];

typedef struct { uint32_t l48, o48, l24, o24, hops; int natural; } Rec;

static Rec walk(const uint8_t* W, const uint16_t* p4, uint32_t p, uint32_t chain, uint32_t nice, uint32_t cap)
{
    uint32_t half = chain >> 1, cl = 2, co = 0, it = 0, d = p4[p], q = p - d, hops = 0;
    uint32_t a24 = 0, b24 = 0;
    int have24 = 0, nat = 0;
    for (;;) {
        if (it >= chain) { nat = 1; break; }
        if (d == 0 || p - q >= 32768) { nat = 1; break; }
        if (hops >= cap) break;
        hops++;
        if (W[q + cl] == W[p + cl] && W[q + cl - 1] == W[p + cl - 1] && W[q + cl - 2] == W[p + cl - 2]) {
            uint32_t m = 0;
            while (m < 258 && W[p + m] == W[q + m]) m++;
            if (m > cl) {
                if (!have24 && it >= half) { a24 = cl; b24 = co; have24 = 1; }
                cl = m; co = p - q;
                if (cl >= nice) { nat = 1; break; }
            }
        }
        it++; d = p4[q]; q -= d;
    }
    if (!have24) { a24 = cl; b24 = co; }
    Rec r = {cl, co, a24, b24, hops, nat};
    return r;
}

/* one lazy parse over rec[]; marks read[] */
static void parse(const Rec* rec, uint32_t len, uint32_t good, uint8_t* read)
{
    uint32_t cur = 0, hm = 0, hl = 0, ho = 0;
    memset(read, 0, len);
    while (cur < len) {
        read[cur] = 1;
        uint32_t rem = len - cur;
        const Rec* r = &rec[cur];
        uint32_t L48 = r->l48 >= 3 ? (r->l48 < rem ? r->l48 : rem) : 0, O48 = r->o48;
        uint32_t L24 = r->l24 >= 3 ? (r->l24 < rem ? r->l24 : rem) : 0, O24 = r->o24;
        if (!hm) {
            uint32_t ml = L48, mo = O48;
            if (ml == 3 && mo > 8192) ml = 2;
            if (ml >= 3) {
                if (ml >= good) cur += ml - 1;
                else { hm = 1; hl = ml; ho = mo; }
            }
        } else {
            uint32_t ml = hl >= 4 ? L24 : L48, mo = hl >= 4 ? O24 : O48;
            int acc = 0;
            if (ml >= hl) { int dl = ml - hl; acc = dl > 4 || (dl * 4 + ilog2(ho) - ilog2(mo)) >= 2; }
            if (acc) { hl = ml; ho = mo; }
            else { cur += hl - 2; hm = 0; }
        }
        cur++;
    }
}

static void block(const uint8_t* blk, uint32_t len, int level, uint32_t cap)
{
    uint32_t good, nice, chain;
    switch (level) {
    case 6: good = 16; nice = 16; chain = 48; break;
    case 7: good = 32; nice = 64; chain = 128; break;
    case 8: good = 64; nice = 128; chain = 320; break;
    default: good = 192; nice = 256; chain = 512;
    }
    uint16_t* p4 = calloc(len + 1, 2);
    int32_t* h4 = malloc(65536 * 4);
    for (int i = 0; i < 65536; i++) h4[i] = -1;
    for (uint32_t p = 0; p < len; p++) {
        uint32_t hd = p ? head_be(blk, p, len) : 0;
        uint32_t a = p ? (hd * 0x1e35a7bdu) >> 16 : 0;
        p4[p] = h4[a] < 0 ? 0 : p - h4[a];
        h4[a] = p;
    }
    uint8_t* W = calloc(len + 600, 1);
    memcpy(W, blk, len);
    Rec* full = malloc(len * sizeof(Rec));
    Rec* cur = malloc(len * sizeof(Rec));
    uint8_t* exact = malloc(len);
    uint8_t* rd = malloc(len);
    for (uint32_t p = 0; p < len; p++) {
        full[p] = walk(W, p4, p, chain, nice, 0xffffffffu);
        cur[p] = walk(W, p4, p, chain, nice, cap);
        exact[p] = cur[p].natural;
        S[1] += full[p].hops;
        S[2] += cur[p].hops;
    }
    int np = 0;
    for (;;) {
        parse(cur, len, good, rd);
        np++;
        uint32_t fixes = 0;
        for (uint32_t p = 0; p < len; p++) {
            const int want = rd[p] || (p && rd[p - 1]);
            if (want && !exact[p]) {
                cur[p] = full[p];
                exact[p] = 1;
                S[3] += full[p].hops;
                fixes++;
            }
        }
        S[4] += fixes;
        if (!fixes || np > 60) break;
    }
    passes_hist[np < 63 ? np : 63]++;
    S[5] += np;
    S[0] += len;
    S[6] += 1;
    free(p4); free(h4); free(W); free(full); free(cur); free(exact); free(rd);
}

int main(int argc, char** argv)
{
    FILE* f = fopen(argv[1], "rb");
    int level = atoi(argv[2]);
    uint32_t cap = argc > 3 ? atoi(argv[3]) : 16;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t* d = malloc(n);
    if (fread(d, 1, n, f) != (size_t) n) return 1;
    for (long o = 0; o < n; o += 65536) block(d + o, (uint32_t) (n - o < 65536 ? n - o : 65536), level, cap);
    double N = S[0];
    printf("level %d cap %u: full hops/pos %.2f | capped pass %.2f + fixes %.2f hops/pos (%.1f fixed positions/block)\n",
           level, cap, S[1] / N, S[2] / N, S[3] / N, S[4] / S[6]);
    printf("  parse passes per block: mean %.2f;", S[5] / S[6]);
    for (int i = 1; i < 64; i++) if (passes_hist[i]) printf(" %d:%.3f", i, passes_hist[i] / S[6]);
    printf("\n");
    return 0;
}
