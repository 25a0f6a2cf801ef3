"""nos_amd.runtime."""
