"""nos_amd.gpu."""
