!======================================================================!
! Fortran `MPI` module interface for amdflang, built from the MPICH
! header that ships in this image (/opt/conda/include/mpif.h).
!
! TEST INFRASTRUCTURE ONLY (oracle/_ref build).  The reference module
! CONTROL (/root/reference/SOURCE/CONTROL.f90:10,83) does `USE MPI` for
! MPI_STATUS_SIZE; the image's mpi.mod is gfortran-format and cannot be
! read by amdflang, so the module is re-formed from MPICH's own include
! file.  No MPI routine is called by the reference hot-path files.
!======================================================================!
MODULE MPI
  IMPLICIT NONE
  INCLUDE 'mpif.h'
END MODULE MPI
