/* kmatch_model.c -- CPU model of k_match's work per position (dev tool, not
 * product).  For each 64 KiB block of a file: the getmatch2 walk with
 * threshold 2 (deflator.c:2650-2674) as k_match runs it, counting hops,
 * quick-reject passes, matchlen 8-byte steps and the reason each walk ends;
 * the positions the lazy parse (compress2 :2826-2906) actually reads; and the
 * hops of a K-gram skip walk (4-chain until the best length reaches K-1, then
 * only candidates sharing K bytes, budget counted by bucket rank).
 *   gcc -O2 -o /tmp/kmm tools/kmatch_model.c && /tmp/kmm file level K
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
static uint32_t lsym(uint32_t len)
{
    uint32_t x = len - 3;
    if (len == 258) return 28;
    if (x < 8) return x;
    uint32_t e = 29 - __builtin_clz(x);
    return 4 * e + 4 + ((x >> e) & 3);
}
static int ilog2(uint32_t x) { return 31 - __builtin_clz(x); }

static double S[32];
static uint64_t hist[600];

static void block(const uint8_t* blk, uint32_t len, int level, uint32_t K)
{
    uint32_t good, nice, chain;
    switch (level) {
    case 6: good = 16; nice = 16; chain = 48; break;
    case 7: good = 32; nice = 64; chain = 128; break;
    case 8: good = 64; nice = 128; chain = 320; break;
    default: good = 192; nice = 256; chain = 512;
    }
    uint32_t half = chain >> 1;
    uint16_t* p4 = calloc(len + 1, 2);
    uint32_t* rank = calloc(len + 1, 4);
    uint32_t* cntb = calloc(65536, 4);
    int32_t* h4 = malloc(65536 * 4);
    for (int i = 0; i < 65536; i++) h4[i] = -1;
    for (uint32_t p = 0; p < len; p++) {
        uint32_t hd = p ? head_be(blk, p, len) : 0;
        uint32_t a = p ? (hd * 0x1e35a7bdu) >> 16 : 0;
        p4[p] = h4[a] < 0 ? 0 : p - h4[a];
        h4[a] = p;
        rank[p] = cntb[a]++;
    }
    uint8_t* W = calloc(len + 600, 1);
    memcpy(W, blk, len);
    /* K-gram chain: previous position with the same K window bytes */
    int32_t* pk = malloc((len + 1) * 4);
    {
        uint32_t HS = 1u << 18;
        int32_t* hk = malloc(HS * 4);
        for (uint32_t i = 0; i < HS; i++) hk[i] = -1;
        for (uint32_t p = 0; p < len; p++) {
            uint64_t h = 1469598103934665603ull;
            for (uint32_t k = 0; k < K; k++) { h ^= W[p + k]; h *= 1099511628211ull; }
            uint32_t s = (uint32_t) (h >> 46);
            int32_t q = hk[s];
            while (q >= 0 && memcmp(W + q, W + p, K) != 0) { s = (s + 1) & (HS - 1); q = hk[s]; }
            pk[p] = q;
            hk[s] = p;
        }
        free(hk);
    }
    uint32_t* hp = malloc(len * 4);       /* hops of each position's full walk */
    uint8_t* nat = malloc(len);            /* walk ended on its own (chain, window, nice) */
    uint32_t* l48 = malloc(len * 4);
    uint32_t* o48 = malloc(len * 4);
    uint32_t* l24 = malloc(len * 4);
    uint32_t* o24 = malloc(len * 4);
    for (uint32_t p = 0; p < len; p++) {
        uint32_t cl = 2, co = 0, it = 0, d = p4[p], q = p - d, why = 0, hops = 0;
        uint32_t a24 = 0, b24 = 0;
        int have24 = 0;
        for (;;) {
            if (it >= chain) { why = 0; break; }
            if (d == 0 || p - q >= 32768) { why = 1; break; }
            hops++;
            S[1]++;
            if (W[q + cl] == W[p + cl] && W[q + cl - 1] == W[p + cl - 1] && W[q + cl - 2] == W[p + cl - 2]) {
                uint32_t m = 0;
                S[2]++;
                while (m < 258 && W[p + m] == W[q + m]) m++;
                S[3] += m / 8 + 1;
                if (m > cl) {
                    S[4]++;
                    if (!have24 && it >= half) { a24 = cl; b24 = co; have24 = 1; }
                    cl = m; co = p - q;
                    if (cl >= nice) { why = 2; break; }
                }
            }
            it++; d = p4[q]; q -= d;
        }
        if (!have24) { a24 = cl; b24 = co; }
        hp[p] = hops;
        nat[p] = why != 0;
        S[5 + why]++;
        hist[hops]++;
        l48[p] = cl; o48[p] = co; l24[p] = a24; o24[p] = b24;
        /* skip walk */
        cl = 2; it = 0; d = p4[p]; q = p - d;
        int onk = 0;
        uint32_t sh = 0;
        for (;;) {
            if (!onk) { if (it >= chain || d == 0 || p - q >= 32768) break; }
            else { if (rank[p] - rank[q] > chain || p - q >= 32768) break; }
            sh++; if (onk) S[12]++;
            if (W[q + cl] == W[p + cl]) {
                uint32_t m = 0;
                while (m < 258 && W[p + m] == W[q + m]) m++;
                if (m > cl) { cl = m; if (cl >= nice) break; }
            }
            if (!onk && cl >= K - 1) onk = 1;
            if (!onk) { it++; d = p4[q]; q -= d; }
            else {
                int32_t qq = (memcmp(W + q, W + p, K) == 0) ? pk[q] : -1;
                if (qq < 0) { qq = pk[p]; while (qq >= 0 && (uint32_t) qq >= q) qq = pk[qq]; }
                if (qq < 0) break;
                q = (uint32_t) qq;
            }
        }
        S[8] += sh;
    }
    /* the lazy parse: which positions are read (compress2 :2826-2906) */
    uint32_t cur = 0, hm = 0, hl = 0, ho = 0, lastc = 0;
    (void) lastc;
    uint8_t* used = calloc(len, 1);
    while (cur < len) {
        used[cur] = 1;
        uint32_t rem = len - cur;
        uint32_t L48 = l48[cur] >= 3 ? (l48[cur] < rem ? l48[cur] : rem) : 0, O48 = o48[cur];
        uint32_t L24 = l24[cur] >= 3 ? (l24[cur] < rem ? l24[cur] : rem) : 0, O24 = o24[cur];
        if (!hm) {
            uint32_t ml = L48, mo = O48;
            if (ml == 3 && mo > 8192) ml = 2;
            if (ml >= 3) {
                if (ml >= good) { S[10]++; cur += ml - 1; }
                else { hm = 1; hl = ml; ho = mo; }
            } else S[11]++;
        } else {
            uint32_t ml = hl >= 4 ? L24 : L48, mo = hl >= 4 ? O24 : O48;
            int acc = 0;
            if (ml >= hl) { int dl = ml - hl; acc = dl > 4 || (dl * 4 + ilog2(ho) - ilog2(mo)) >= 2; }
            if (acc) { S[11]++; hl = ml; ho = mo; }
            else { S[10]++; cur += hl - 2; hm = 0; }
        }
        cur++;
    }
    for (uint32_t p = 0; p < len; p++) S[9] += used[p];
    /* capped first pass: hops min(h, C) everywhere, plus the full walk again
     * at read positions (and the position after each) whose walk the cap
     * truncated (not ended on its own within C hops) */
    {
        static const uint32_t CAPS[4] = {8, 16, 32, 64};
        for (int c = 0; c < 4; c++) {
            uint32_t C = CAPS[c];
            double h1 = 0, h2 = 0, nt = 0;
            for (uint32_t p = 0; p < len; p++) {
                h1 += hp[p] < C ? hp[p] : C;
                const int trunc = hp[p] >= C && !(nat[p] && hp[p] <= C);
                const int rd = used[p] || (p && used[p - 1]);
                if (trunc && rd) { h2 += hp[p]; nt++; }
            }
            S[16 + 3 * c] += h1;
            S[17 + 3 * c] += h2;
            S[18 + 3 * c] += nt;
        }
    }
    free(hp); free(nat);
    S[0] += len;
    free(used); free(l48); free(o48); free(l24); free(o24);
    free(p4); free(rank); free(cntb); free(h4); free(W); free(pk);
    (void) lsym;
}

int main(int argc, char** argv)
{
    FILE* f = fopen(argv[1], "rb");
    int level = atoi(argv[2]);
    uint32_t K = argc > 3 ? atoi(argv[3]) : 6;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t* d = malloc(n);
    if (fread(d, 1, n, f) != (size_t) n) return 1;
    for (long o = 0; o < n; o += 65536) block(d + o, (uint32_t) (n - o < 65536 ? n - o : 65536), level, K);
    double N = S[0];
    printf("positions %.0f\n hops/pos %.2f  passes/pos %.2f  ml8steps/pos %.2f  improves/pos %.2f\n",
           N, S[1] / N, S[2] / N, S[3] / N, S[4] / N);
    printf(" end: budget %.3f  chain/dist %.3f  nice %.3f\n", S[5] / N, S[6] / N, S[7] / N);
    printf(" skip(K=%u) hops/pos %.2f (of which K-chain %.2f)\n", K, S[8] / N, S[12] / N);
    printf(" parse reads %.3f of positions (matches %.0f literals %.0f per block)\n", S[9] / N,
           S[10] / (N / 65536), S[11] / (N / 65536));
    {
        static const uint32_t CAPS[4] = {8, 16, 32, 64};
        for (int c = 0; c < 4; c++)
            printf(" cap %2u: pass1 hops/pos %.2f  fix hops/pos %.2f  truncated read pos/block %.1f\n", CAPS[c],
                   S[16 + 3 * c] / N, S[17 + 3 * c] / N, S[18 + 3 * c] / (N / 65536));
    }
    printf(" hops hist:");
    for (int i = 0; i <= 48; i += 4) {
        uint64_t s = 0;
        for (int j = i; j < i + 4 && j < 600; j++) s += hist[j];
        printf(" %d:%.3f", i, s / N);
    }
    uint64_t s = 0;
    for (int j = 52; j < 600; j++) s += hist[j];
    printf(" 52+:%.3f\n", s / N);
    return 0;
}
