"""nos_amd.resource."""
