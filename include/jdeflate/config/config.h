/*
 * jdeflate/config/config.h -- export macro and version for the MI355X
 * jdeflate engine.  Replaces the meson-generated header of the reference
 * (jdeflate/config/config.h.in:29-75); same macro names.
 */
#ifndef JDEFLATE_CONFIG_H
#define JDEFLATE_CONFIG_H

#include <jdeflate/config/types.h>

#ifndef JDEFLATE_API
	#if defined(__GNUC__)
		#define JDEFLATE_API __attribute__((visibility("default")))
	#else
		#define JDEFLATE_API
	#endif
#endif

#define JDEFLATE_VERSION_MAJOR 0
#define JDEFLATE_VERSION_MINOR 4
#define JDEFLATE_VERSION_PATCH 0
#define JDEFLATE_VERSION_STRING "0.4.0-mi355x"

struct JDEFLATEVersion {
	int major;
	int minor;
	int patch;
	const char* versionstring;
	const char* builddate;
};

#ifdef __cplusplus
extern "C" {
#endif

/* version.c:23-35 */
JDEFLATE_API struct JDEFLATEVersion jdeflate_getversion(void);

#ifdef __cplusplus
}
#endif

#endif
