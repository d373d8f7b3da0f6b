# Generates OpenFHE's config_core.h from the reference's OWN template
# (configure/config_core.in) with the values the reference's CMakeLists.txt
# sets by default -- the same configure_file() call as CMakeLists.txt:365,
# run in script mode (no project configure, no build system).
#
#   cmake -DSRC=<ref>/configure/config_core.in -DDST=<out>/config_core.h -P ref_config_core.cmake
#
# Values (CMakeLists.txt line):
#   WITH_BE2 ON, WITH_BE4 ON, WITH_NTL OFF, WITH_TCM OFF          (:85-88)
#   NATIVE_SIZE 64 -> NATIVEINT 64                                 (:95-97, :302-305)
#   HAVE_INT128 / HAVE_INT64 = TRUE (check_type_size on x86-64)    (:284-286)
#   MATHBACKEND 4                                                  (:326-328)
#   CKKS_M_FACTOR 1                                                (:100-101)
set(WITH_BE2 ON)
set(WITH_BE4 ON)
set(WITH_NTL OFF)
set(WITH_TCM OFF)
set(MATHBACKEND 4)
set(HAVE_INT128 TRUE)
set(HAVE_INT64 TRUE)
set(NATIVEINT 64)
set(CKKS_M_FACTOR 1)
if(NOT SRC OR NOT DST)
  message(FATAL_ERROR "usage: cmake -DSRC=... -DDST=... -P ref_config_core.cmake")
endif()
configure_file(${SRC} ${DST})
