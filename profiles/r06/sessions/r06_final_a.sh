TAG=r06fa STEPS="tests smoke bench rocprof pipeline" PIPE_CONFIGS="tsp1080 dof4k" bash tools/session.sh && TAG=r06fa STEPS="pmc" CONFIGS="tsp1080 blob1080" bash tools/session.sh
