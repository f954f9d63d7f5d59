#!/bin/bash
# RStudio session wrapper: the session inherits the container's environment (NB_PREFIX, proxies,
# HIP/ROCm variables) the way the reference's rsession.sh hands it through.
export USER="${NB_USER:-jovyan}"
exec /usr/lib/rstudio-server/bin/rsession "$@"
