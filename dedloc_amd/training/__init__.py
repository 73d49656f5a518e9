"""dedloc_amd.training"""
