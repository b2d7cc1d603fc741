      ****************************************************************************
      *                                                                          *
      * Copyright 2018 ABSA Group Limited                                        *
      *                                                                          *
      * Licensed under the Apache License, Version 2.0 (the "License");          *
      * you may not use this file except in compliance with the License.         *
      * You may obtain a copy of the License at                                  *
      *                                                                          *
      *     http://www.apache.org/licenses/LICENSE-2.0                           *
      *                                                                          *
      * Unless required by applicable law or agreed to in writing, software      *
      * distributed under the License is distributed on an "AS IS" BASIS,        *
      * WITHOUT WARRANTIES OR CONDITIONS OF ANY KIND, either express or implied. *
      * See the License for the specific language governing permissions and      *
      * limitations under the License.                                           *
      *                                                                          *
      ****************************************************************************

      01 RECORD.
          02 COUNT PIC 9(1).
          02 GROUP OCCURS 0 TO 2 TIMES DEPENDING ON COUNT.
             03 INNER-COUNT PIC 9(1).
             03 INNER-GROUP OCCURS 0 TO 3 TIMES
                                DEPENDING ON INNER-COUNT.
                04 FIELD PIC X.
