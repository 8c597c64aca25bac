# Writes OUT (a one-line header defining STENCIL_GIT_SHA) from `git describe` of SRC; rewritten only when the
# revision or the dirty state changes, so an unchanged tree rebuilds nothing. Reference equivalent:
# cmake/GetGitRevisionDescription.cmake (git hash embedded in the binaries).
execute_process(COMMAND git -C ${SRC} rev-parse --short=12 HEAD OUTPUT_VARIABLE sha
                OUTPUT_STRIP_TRAILING_WHITESPACE ERROR_QUIET RESULT_VARIABLE rc)
if(NOT rc EQUAL 0 OR sha STREQUAL "")
  set(sha "unknown")
else()
  execute_process(COMMAND git -C ${SRC} status --porcelain --untracked-files=no OUTPUT_VARIABLE dirty
                  OUTPUT_STRIP_TRAILING_WHITESPACE ERROR_QUIET)
  if(NOT dirty STREQUAL "")
    set(sha "${sha}-dirty")
  endif()
endif()
set(text "#define STENCIL_GIT_SHA \"${sha}\"\n")
if(EXISTS ${OUT})
  file(READ ${OUT} old)
else()
  set(old "")
endif()
if(NOT old STREQUAL text)
  file(WRITE ${OUT} "${text}")
endif()
