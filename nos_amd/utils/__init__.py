"""nos_amd.utils."""
