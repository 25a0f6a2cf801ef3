"""Node-local agents: the partition agent (``migagent`` analogue), the
CU-mask gpuagent and the node labeler (the GPU operator's feature discovery
role), plus the state they share."""
