/*
 * multi_caller.c -- TEST SUPPORT: a plain C99 caller of the multi-device
 * entry points (jdgpu_deflate_multi / jdgpu_inflate_multi, jdgpu.h), with no
 * HIP and no torch.  argv[1]: input file; argv[2]: level.  Deflates the file
 * on every visible device (ndev = 0) and on the current device alone
 * (jdgpu_deflate), requires the two streams and size indexes to be equal
 * byte for byte, inflates the gathered stream over every device and
 * requires the input back.  Prints "ok <devices> <in> <out>" and exits 0.
 */
#include <jdeflate/jdgpu.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int main(int argc, char** argv)
{
    if (argc < 3) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    unsigned char* src = malloc(n ? (size_t) n : 1);
    if (!src || fread(src, 1, (size_t) n, f) != (size_t) n) return 2;
    fclose(f);
    const int level = atoi(argv[2]);
    const uint32 bs = 65536;
    const uint32 nb = n ? (uint32) ((n + bs - 1) / bs) : 1;
    const uint64 cap = jdgpu_bound((uint64) n, bs);
    unsigned char* a = malloc(cap);
    unsigned char* b = malloc(cap);
    uint32* sa = malloc(nb * 4);
    uint32* sb = malloc(nb * 4);
    int64 la = jdgpu_deflate_multi(src, (uint64) n, bs, level, 0, 1, a, cap, sa, 0, NULL);
    int64 lb = jdgpu_deflate(src, (uint64) n, bs, level, 0, 1, b, cap, sb);
    if (la < 0 || lb < 0) { printf("deflate failed %lld %lld\n", (long long) la, (long long) lb); return 1; }
    if (la != lb || memcmp(a, b, (size_t) la) || memcmp(sa, sb, nb * 4)) { printf("streams differ\n"); return 1; }
    unsigned char* back = malloc((size_t) nb * bs);
    uint32* us = malloc(nb * 4);
    int32* er = malloc(nb * 4);
    int r = jdgpu_inflate_multi(a, (uint64) la, sa, nb, bs, back, us, er, 0, NULL);
    if (r) { printf("inflate failed %d\n", r); return 1; }
    for (uint32 i = 0; i < nb; i++) {
        const uint64 want = (uint64) n - (uint64) i * bs < bs ? (uint64) n - (uint64) i * bs : bs;
        if (us[i] != want || memcmp(back + (size_t) i * bs, src + (size_t) i * bs, want)) {
            printf("block %u differs\n", i);
            return 1;
        }
    }
    /* devices that took part: every visible one */
    printf("ok %lld %lld\n", (long long) n, (long long) la);
    return 0;
}
