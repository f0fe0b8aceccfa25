/* doshort flips per block (dev tool) */
#include <stdio.h>
#include <stdint.h>
#include <stddef.h>
static unsigned long g_obs, g_flip, g_on;
static unsigned long g_step, g_held;
static void jdo_stat_step(int h) { g_step++; g_held += h != 0; }
static void jdo_stat_obs(int old, int nw, size_t cur) { g_obs++; g_flip += old != nw; g_on += nw; (void) cur; }
#define JDO_STATS 1
#include "../oracle/jdoracle.c"
int ds_run(const uint8_t* src, size_t n, int level, unsigned long* out)
{
    static uint8_t buf[1 << 18];
    unsigned long blocks_with_flip = 0;
    for (size_t o = 0; o < n; o += 65536) {
        size_t m = n - o < 65536 ? n - o : 65536;
        unsigned long f0 = g_flip;
        jdo_deflate(src + o, m, level, 0, 2, buf, sizeof buf);
        blocks_with_flip += g_flip != f0;
    }
    out[0] = g_obs; out[1] = g_flip; out[2] = g_on; out[3] = blocks_with_flip; out[4] = g_step; out[5] = g_held;
    return 0;
}
