"""nos_amd.cmd."""
