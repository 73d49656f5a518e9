// Host-only stand-in for the two HIP runtime calls comm_core.cpp makes (device switching).
#pragma once
typedef enum { hipSuccess = 0, hipErrorInvalidDevice = 101 } hipError_t;
hipError_t hipGetDevice(int* dev);
hipError_t hipSetDevice(int dev);
