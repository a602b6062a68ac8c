/*
 * mpcr_mjcf.h -- C ABI of libmpcr_mjcf.so, the MJCF -> mpcr_model_t compiler
 * (MjModel.from_xml_path, SBP/mjx_planner.py:100-103).  mpcr_model_load
 * (mpcr.h) calls it for .xml paths; hosts that want the serialised model
 * itself (to cache or ship it) call it directly and pass the blob to
 * mpcr_model_from_blob.
 *
 * The compiler is manipulator_mujoco_amd/mjcf.py run in an embedded CPython
 * (started on first use when the host has none; the package root is found
 * next to the library).  One compile at a time (internally serialised).
 */
#ifndef MPCR_MJCF_H_
#define MPCR_MJCF_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Compile the MJCF at path (timestep <= 0: the file's <option timestep>).
   On success *blob is a malloc'd mpcr_model_t of *nbytes bytes (release it
   with mpcr_mjcf_free) and 0 is returned; on failure -1 and a message in
   err[errlen]. */
int mpcr_mjcf_compile(const char* path, double timestep, void** blob, size_t* nbytes, char* err, int errlen);
void mpcr_mjcf_free(void* blob);

#ifdef __cplusplus
}
#endif

#endif /* MPCR_MJCF_H_ */
