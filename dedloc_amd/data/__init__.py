"""dedloc_amd.data"""
