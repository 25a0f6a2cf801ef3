"""nos_amd.sim."""
