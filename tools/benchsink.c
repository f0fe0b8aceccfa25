/* bench.py helper (not the product): a zstrm write callback in C that
 * appends to a caller buffer, so zstrm_gzip_pcie times the library and not
 * a Python callback per 32 KiB write */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

typedef struct {
    uint8_t* base;
    size_t cap, pos;
} BenchSink;

intptr_t bench_sink_write(const uint8_t* buf, size_t size, void* user)
{
    BenchSink* s = (BenchSink*) user;
    if (s->pos + size > s->cap) return -1;
    memcpy(s->base + s->pos, buf, size);
    s->pos += size;
    return (intptr_t) size;
}
