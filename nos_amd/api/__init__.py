"""nos_amd.api."""
