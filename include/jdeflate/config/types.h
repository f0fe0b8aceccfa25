/*
 * jdeflate/config/types.h -- the ctoolbox vocabulary the public headers use.
 *
 * When the real ctoolbox headers are on the include path (as they are for
 * applications built against the reference), they are used as-is so the
 * types are identical.  Otherwise minimal equivalents are defined here:
 * uintxx/intxx are pointer-sized, TAllocator is
 * {request, dispose, user} as called in deflator.c:283/526 and
 * inflator.c:174/258.
 */
#ifndef JDEFLATE_TYPES_H
#define JDEFLATE_TYPES_H

#if defined(__has_include)
	#if __has_include(<ctoolbox/ctoolbox.h>) && __has_include(<ctoolbox/memory.h>) && !defined(JDEFLATE_NO_CTOOLBOX)
		#define JDEFLATE_HAVE_CTOOLBOX 1
	#endif
#endif

#if defined(JDEFLATE_HAVE_CTOOLBOX)
	#include <ctoolbox/ctoolbox.h>
	#include <ctoolbox/memory.h>
#else
	#include <stddef.h>
	#include <stdint.h>
	#include <assert.h>
	#if !defined(__cplusplus)
		#include <stdbool.h>
	#endif

typedef uint8_t  uint8;
typedef uint16_t uint16;
typedef uint32_t uint32;
typedef uint64_t uint64;
typedef int16_t  int16;
typedef int32_t  int32;
typedef int64_t  int64;
typedef uintptr_t uintxx;
typedef intptr_t  intxx;

	#if defined(__cplusplus)
		#define CTB_INLINE static inline
	#else
		#define CTB_INLINE static inline
	#endif
	#define CTB_FORCEINLINE CTB_INLINE
	#if defined(__GNUC__)
		#define CTB_EXPECT0(x) __builtin_expect(!!(x), 0)
		#define CTB_EXPECT1(x) __builtin_expect(!!(x), 1)
	#else
		#define CTB_EXPECT0(x) (x)
		#define CTB_EXPECT1(x) (x)
	#endif
	#define CTB_ASSERT(x) assert(x)

struct TAllocator {
	void* (*request)(uintxx size, void* user);
	void  (*dispose)(void* memory, uintxx size, void* user);
	void* user;
};
typedef struct TAllocator TAllocator;
#endif

#endif
