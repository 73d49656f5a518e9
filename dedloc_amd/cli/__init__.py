"""dedloc_amd.cli"""
