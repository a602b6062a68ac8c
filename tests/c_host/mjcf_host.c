/* A non-Python host of the C ABI: loads a scene from its MJCF through
   mpcr_model_load (the replacement for MjModel.from_xml_path,
   SBP/mjx_planner.py:100-103) and prints the model's sizes.  Built and run by
   tests/test_lib.py::test_c_host_loads_mjcf (no GPU needed).
     mjcf_host <libmpcr.so> <scene.xml> <timestep>                        */
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>

typedef struct mpcr_model mpcr_model;

int main(int argc, char** argv) {
  if (argc < 4) return 2;
  void* so = dlopen(argv[1], RTLD_NOW);
  if (!so) { fprintf(stderr, "dlopen: %s\n", dlerror()); return 3; }
  int (*load)(const char*, double, mpcr_model**) = (int (*)(const char*, double, mpcr_model**))dlsym(so, "mpcr_model_load");
  int (*info)(const mpcr_model*, int*, int*, int*, int*, int*) =
      (int (*)(const mpcr_model*, int*, int*, int*, int*, int*))dlsym(so, "mpcr_model_info");
  void (*release)(mpcr_model*) = (void (*)(mpcr_model*))dlsym(so, "mpcr_model_free");
  const char* (*last_error)(void) = (const char* (*)(void))dlsym(so, "mpcr_last_error");
  if (!load || !info || !release || !last_error) return 4;
  mpcr_model* m = NULL;
  int rc = load(argv[2], atof(argv[3]), &m);
  if (rc) { fprintf(stderr, "mpcr_model_load: %d %s\n", rc, last_error()); return 5; }
  int nq, nv, nslot, nctrl, npair;
  if (info(m, &nq, &nv, &nslot, &nctrl, &npair)) return 6;
  printf("nq=%d nv=%d nslot=%d nctrl=%d npair=%d\n", nq, nv, nslot, nctrl, npair);
  release(m);
  return 0;
}
